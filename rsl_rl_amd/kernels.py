"""Tensor-level wrappers over the C ABI (include/rslrl_amd.h) -- the hot path's Python face.

Every device entry point takes torch tensors that live on a ROCm device, launches on the current
torch stream and never synchronises.  CPU tensors are rejected: there is no CPU fallback.
"""

from __future__ import annotations

import contextlib
import ctypes
from collections import defaultdict

import torch

from . import _lib

__all__ = [
    "compute_returns",
    "compute_returns_records",
    "normalize_advantages_",
    "randperm_mt19937",
    "gather_rows",
    "gather_records",
    "record_fill_slot",
    "ppo_loss_fwd_bwd",
    "PPOLossFunction",
    "rollout_record",
]


def _require_device(*tensors: torch.Tensor):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "rsl_rl_amd: the PPO hot path runs only on a ROCm GPU (torch 'cuda' device); got a tensor "
                f"on {t.device}. There is no CPU fallback."
            )


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _Workspace:
    """Per-(device, purpose) scratch buffers from torch's caching allocator, grown on demand.

    Reuse across calls is stream-ordered (all launches go to the current stream of the device).
    """

    def __init__(self):
        self._bufs = {}

    def get(self, device: torch.device, key: str, nbytes: int) -> torch.Tensor:
        # zero-filled on allocation: the loss workspace begins with an arrival counter that the library
        # expects to be zero before its first use and leaves zero after every call
        k = (device, key)
        buf = self._bufs.get(k)
        if buf is None or buf.numel() < nbytes:
            buf = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)
            self._bufs[k] = buf
        return buf


_ws = _Workspace()


_NO_SPAN = contextlib.nullcontext()


class KernelTimer:
    """Optional HIP-event timing of each C-ABI call, recorded on the stream the kernels launch on.

    bench.py enables it over its timed region to report the dominant kernel's live launch duration
    (roofline.achieved); disabled it costs one attribute check per call.
    """

    def __init__(self):
        self.enabled = False
        self.mlp_enabled = False  # the (many) MLP GEMM launches are timed separately from the hot path
        self.spans = defaultdict(list)
        self.bytes = defaultdict(list)
        self.flops = defaultdict(list)

    def reset(self):
        self.spans.clear()
        self.bytes.clear()
        self.flops.clear()

    def span(self, name: str, device: torch.device, algorithmic_bytes: int, flops: int = 0):
        # disabled (every call outside bench.py's timed region): one shared no-op context, no generator per call
        if not (self.mlp_enabled if name.startswith("linear_") else self.enabled):
            return _NO_SPAN
        return self._span(name, device, algorithmic_bytes, flops)

    @contextlib.contextmanager
    def _span(self, name: str, device: torch.device, algorithmic_bytes: int, flops: int = 0):
        stream = torch.cuda.current_stream(device)
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record(stream)
        yield
        end.record(stream)
        self.spans[name].append((start, end))
        self.bytes[name].append(algorithmic_bytes)
        self.flops[name].append(flops)

    # launches of the loss kernel, the rollout record and the record gather bound to their own event pair inside the
    # library (rslrl_launch_timing_*, one tag per kernel): the dispatch's begin-to-end time, the duration rocprofv3
    # reports, next to the marker span of the C-ABI call
    def arm_launch_events(self, capacity: int = 4096):
        _lib.check(_lib.lib().rslrl_launch_timing_enable(capacity), "rslrl_launch_timing_enable")

    def disarm_launch_events(self):
        _lib.check(_lib.lib().rslrl_launch_timing_enable(0), "rslrl_launch_timing_enable")

    LAUNCH_TAGS = {"ppo_loss": _lib.LAUNCH_TAG_PPO_LOSS, "rollout_record": _lib.LAUNCH_TAG_ROLLOUT_RECORD,
                   "gather_rows": _lib.LAUNCH_TAG_GATHER_RECORDS}

    @staticmethod
    def launch_events(kernel: str = "ppo_loss"):
        """(total_ms, launches) of `kernel`'s launches bound to events since the last arm_launch_events()."""
        ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
        tag = KernelTimer.LAUNCH_TAGS[kernel]
        _lib.check(_lib.lib().rslrl_launch_timing_read_tag(tag, ctypes.byref(ms), ctypes.byref(n)),
                   "rslrl_launch_timing_read_tag")
        return ms.value, n.value

    def summary(self):
        """name -> {launches, mean_ms, total_ms, bytes_per_launch}; synchronises the events."""
        out = {}
        for name, evs in self.spans.items():
            ms = [s.elapsed_time(e) for s, e in evs]
            out[name] = {
                "launches": len(ms),
                "mean_ms": sum(ms) / len(ms),
                "total_ms": sum(ms),
                "bytes_per_launch": sum(self.bytes[name]) / len(self.bytes[name]),
                "flops_per_launch": sum(self.flops[name]) / len(self.flops[name]),
            }
        return out


timer = KernelTimer()


def normal_affine_(x: torch.Tensor, scale: torch.Tensor, loc: torch.Tensor) -> torch.Tensor:
    """x <- x * scale + loc in place (torch's mul_ then add_ roundings) in one launch (rslrl_normal_affine): the
    rollout's Normal sample from standard normals x [N, A] contiguous; scale / loc [N, A] with unit column stride
    (row stride 0 for an expanded shared std)."""
    _require_device(x, scale, loc)
    if x.dim() != 2 or not x.is_contiguous() or scale.shape != x.shape or loc.shape != x.shape:
        raise ValueError("normal_affine_: x [N, A] contiguous, scale / loc of its shape")
    if (scale.stride(1) != 1 and x.shape[1] > 1) or (loc.stride(1) != 1 and x.shape[1] > 1):
        raise ValueError("normal_affine_: scale / loc need unit column stride")
    N, A = x.shape
    rc = _lib.lib().rslrl_normal_affine(x.data_ptr(), scale.data_ptr(), scale.stride(0), loc.data_ptr(), loc.stride(0),
                                        N, A, ctypes.c_void_p(_stream(x.device)))
    _lib.check(rc, "rslrl_normal_affine")
    return x


# ------------------------------------------------------------------------------------------------
# rollout_storage.py:127-149
# ------------------------------------------------------------------------------------------------
def _gae_workspace(dev: torch.device, T: int, N: int) -> torch.Tensor:
    """compute_returns' workspace of the current stream: the one-launch forms keep a grid barrier's ticket in it, so two
    streams must not share one (include/rslrl_amd.h, ABI 18)."""
    return _ws.get(dev, ("gae", _stream(dev)), _lib.lib().rslrl_compute_returns_workspace_bytes(T, N))


def gae_status_word(ws: torch.Tensor) -> torch.Tensor:
    """The workspace's uint32 grid-barrier status word as a 1-element int32 device view (0 = ok)."""
    off = _lib.lib().rslrl_compute_returns_status_offset()
    return ws[off:off + 4].view(torch.int32)


class GAEBarrierTimeout(RuntimeError):
    """compute_returns' one-launch grid barrier timed out: its blocks were not co-resident (another kernel or process
    held CUs), so that call's advantages are NaN."""


def raise_on_gae_status(status: torch.Tensor, value: float | int | None = None) -> None:
    """Raise GAEBarrierTimeout if the status word (or its already read-back `value`) is set; clears the word."""
    v = int(status.item()) if value is None else int(value)
    if v != 0:
        with torch.inference_mode():  # the word may be a view made under the runner's inference mode
            status.zero_()
        raise GAEBarrierTimeout(
            "rsl_rl_amd compute_returns: the one-launch GAE's grid barrier timed out (its blocks were not all resident "
            "at once), so the advantages of that rollout are NaN; set RSLRL_GAE_FUSED=0 to use the two-launch form")


def debug_knob(name: str, value: int) -> int:
    """Set one of the library's test knobs (include/rslrl_amd.h rslrl_debug_knob); returns the previous value."""
    prev = ctypes.c_int64(0)
    _lib.check(_lib.lib().rslrl_debug_knob(name.encode(), int(value), ctypes.byref(prev)), "rslrl_debug_knob")
    return prev.value


def compute_returns(values, rewards, dones, last_values, gamma, lam, normalize_advantage, returns, advantages):
    """GAE + (optional) normalisation, written into `returns` / `advantages` ([T, N, 1] fp32, in place).

    values/rewards [T, N, 1] fp32, dones [T, N, 1] uint8, last_values [N, 1] fp32, all contiguous.
    """
    _require_device(values, rewards, dones, last_values, returns, advantages)
    T, N = values.shape[0], values.shape[1]
    for t, dt in ((values, torch.float32), (rewards, torch.float32), (dones, torch.uint8),
                  (last_values, torch.float32), (returns, torch.float32), (advantages, torch.float32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"compute_returns: expected contiguous {dt}, got {t.dtype} (contiguous={t.is_contiguous()})")
    if values.numel() != T * N or last_values.numel() != N or dones.numel() != T * N or rewards.numel() != T * N:
        raise ValueError("compute_returns: inconsistent shapes")
    L = _lib.lib()
    dev = values.device
    ws = _gae_workspace(dev, T, N)
    # one span over the production entry point (scan + fused normalisation): algorithmic bytes of both passes
    moved = 17 * T * N + 4 * N + (8 * T * N if normalize_advantage else 0)
    with timer.span("compute_returns", dev, moved):
        rc = L.rslrl_compute_returns(
            _ptr(values), _ptr(rewards), _ptr(dones), _ptr(last_values), ctypes.c_float(gamma), ctypes.c_float(lam),
            T, N, int(bool(normalize_advantage)), _ptr(returns), _ptr(advantages), _ptr(ws),
            ws.numel(), ctypes.c_void_p(_stream(dev)),
        )
    _lib.check(rc, "rslrl_compute_returns")


def compute_returns_records(values, rewards, dones, last_values, gamma, lam, returns, advantages, log_prob, records,
                            slot_offset: int):
    """compute_returns with normalisation whose last pass also writes every record's slot
    {value, log-prob, return, advantage, 0, 0, 0, 0} at `slot_offset` (include/rslrl_amd.h
    rslrl_compute_returns_records): records [T, N, R] contiguous fp32, log_prob [T, N, 1] contiguous fp32."""
    _require_device(values, rewards, dones, last_values, returns, advantages, log_prob, records)
    T, N = values.shape[0], values.shape[1]
    for t, dt in ((values, torch.float32), (rewards, torch.float32), (dones, torch.uint8), (last_values, torch.float32),
                  (returns, torch.float32), (advantages, torch.float32), (log_prob, torch.float32),
                  (records, torch.float32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"compute_returns_records: expected contiguous {dt}, got {t.dtype} "
                             f"(contiguous={t.is_contiguous()})")
    if (values.numel() != T * N or last_values.numel() != N or dones.numel() != T * N or rewards.numel() != T * N
            or log_prob.numel() != T * N or records.dim() != 3 or records.shape[:2] != values.shape[:2]):
        raise ValueError("compute_returns_records: inconsistent shapes")
    R = records.shape[2]
    L = _lib.lib()
    dev = values.device
    ws = _gae_workspace(dev, T, N)
    # scan (17 B + 4 B per env) + normalisation reading adv / value / log-prob / return and writing adv + the slot
    moved = 17 * T * N + 4 * N + (4 * 4 + 4 + 32) * T * N
    with timer.span("compute_returns", dev, moved):
        rc = L.rslrl_compute_returns_records(
            _ptr(values), _ptr(rewards), _ptr(dones), _ptr(last_values), ctypes.c_float(gamma), ctypes.c_float(lam),
            T, N, _ptr(returns), _ptr(advantages), _ptr(log_prob), _ptr(records), R, int(slot_offset), _ptr(ws),
            ws.numel(), ctypes.c_void_p(_stream(dev)),
        )
    _lib.check(rc, "rslrl_compute_returns_records")


def compute_returns_slots(values, rewards, dones, last_values, gamma, lam, returns, advantages, log_prob, slots):
    """compute_returns with normalisation whose last pass also writes the scalar slot array
    slots[t, n] = {value, log-prob, return, advantage} (include/rslrl_amd.h rslrl_compute_returns_slots): slots
    [T, N, 4] contiguous fp32, log_prob [T, N, 1] contiguous fp32.  Returns the workspace's barrier status word (a
    1-element int32 device tensor, read it with raise_on_gae_status at the next synchronisation)."""
    _require_device(values, rewards, dones, last_values, returns, advantages, log_prob, slots)
    T, N = values.shape[0], values.shape[1]
    for t, dt in ((values, torch.float32), (rewards, torch.float32), (dones, torch.uint8), (last_values, torch.float32),
                  (returns, torch.float32), (advantages, torch.float32), (log_prob, torch.float32),
                  (slots, torch.float32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"compute_returns_slots: expected contiguous {dt}, got {t.dtype} "
                             f"(contiguous={t.is_contiguous()})")
    if (values.numel() != T * N or last_values.numel() != N or dones.numel() != T * N or rewards.numel() != T * N
            or log_prob.numel() != T * N or slots.numel() != 4 * T * N):
        raise ValueError("compute_returns_slots: inconsistent shapes")
    L = _lib.lib()
    dev = values.device
    ws = _gae_workspace(dev, T, N)
    form = L.rslrl_compute_returns_slots_form(T, N, _ptr(values), _ptr(rewards), _ptr(dones), _ptr(log_prob),
                                              _ptr(returns), _ptr(advantages))
    if form != 0:
        # the one-launch forms (ABI 16 / 18): read value, reward, done, log-prob (13 B) + last value per env, write
        # return, advantage and the 16-byte slot (24 B)
        moved = 37 * T * N + 4 * N
    else:
        # scan (17 B + 4 B per env) + normalisation reading adv / value / log-prob / return, writing adv + the slot
        moved = 17 * T * N + 4 * N + (4 * 4 + 4 + 16) * T * N
    with timer.span("compute_returns", dev, moved):
        rc = L.rslrl_compute_returns_slots(
            _ptr(values), _ptr(rewards), _ptr(dones), _ptr(last_values), ctypes.c_float(gamma), ctypes.c_float(lam),
            T, N, _ptr(returns), _ptr(advantages), _ptr(log_prob), _ptr(slots), _ptr(ws), ws.numel(),
            ctypes.c_void_p(_stream(dev)),
        )
    _lib.check(rc, "rslrl_compute_returns_slots")
    return gae_status_word(ws)


def normalize_advantages_(adv: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """In-place (adv - mean) / (std_unbiased + eps) over all elements (rollout_storage.py:149)."""
    _require_device(adv)
    if adv.dtype != torch.float32 or not adv.is_contiguous():
        raise ValueError("normalize_advantages_: expected a contiguous fp32 tensor")
    L = _lib.lib()
    n = adv.numel()
    ws = _ws.get(adv.device, "norm", L.rslrl_normalize_workspace_bytes(n))
    with timer.span("adv_normalize", adv.device, 12 * n):
        rc = L.rslrl_normalize_advantages(_ptr(adv), n, ctypes.c_float(eps), _ptr(ws), ws.numel(),
                                          ctypes.c_void_p(_stream(adv.device)))
    _lib.check(rc, "rslrl_normalize_advantages")
    return adv


# ------------------------------------------------------------------------------------------------
# rollout_storage.py:165 -- torch CPU randperm semantics, host mt19937
# ------------------------------------------------------------------------------------------------
def randperm_mt19937(n: int, generator: torch.Generator | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Exactly torch.randperm(n, generator=generator) for a CPU generator (default: the process default
    CPU generator), returned as int32 and advancing the generator identically.  Host code."""
    gen = torch.default_generator if generator is None else generator
    if gen.device.type != "cpu":
        raise ValueError("randperm_mt19937 follows torch's CPU generator; pass a CPU torch.Generator")
    state = gen.get_state()
    if out is None:
        out = torch.empty(n, dtype=torch.int32)
    if out.dtype != torch.int32 or out.device.type != "cpu" or not out.is_contiguous() or out.numel() < n:
        raise ValueError("randperm_mt19937: `out` must be a contiguous CPU int32 tensor with >= n elements")
    rc = _lib.lib().rslrl_randperm_mt19937(_ptr(state), state.numel(), n, _ptr(out))
    _lib.check(rc, "rslrl_randperm_mt19937")
    gen.set_state(state)
    return out[:n]


def randperm_mt19937_state(n: int, state: torch.Tensor, out: torch.Tensor) -> None:
    """randperm_mt19937 on a CPU generator-state blob (torch.Generator.get_state()) instead of a generator:
    writes the permutation into `out` (contiguous CPU int32, >= n elements) and advances `state` in place to
    what the generator's state would be afterwards.  Touches no torch state, so it may run on a worker thread
    (ctypes releases the GIL for the call)."""
    if out.dtype != torch.int32 or out.device.type != "cpu" or not out.is_contiguous() or out.numel() < n:
        raise ValueError("randperm_mt19937_state: `out` must be a contiguous CPU int32 tensor with >= n elements")
    rc = _lib.lib().rslrl_randperm_mt19937(_ptr(state), state.numel(), n, _ptr(out))
    _lib.check(rc, "rslrl_randperm_mt19937")


# ------------------------------------------------------------------------------------------------
# rollout_storage.py:168-197 -- all mini-batch fields in one launch
# ------------------------------------------------------------------------------------------------
def gather_rows(pairs, indices: torch.Tensor):
    """pairs: list of (src [rows, ...], dst [count, ...]) contiguous tensors; dst[r] = src[indices[r]]."""
    if len(pairs) > _lib.MAX_GATHER_FIELDS:
        for i in range(0, len(pairs), _lib.MAX_GATHER_FIELDS):
            gather_rows(pairs[i:i + _lib.MAX_GATHER_FIELDS], indices)
        return
    _require_device(indices, *[t for p in pairs for t in p])
    if indices.dtype != torch.int32 or not indices.is_contiguous():
        raise ValueError("gather_rows: indices must be contiguous int32")
    count = indices.numel()
    arr = (_lib.GatherField * max(len(pairs), 1))()
    moved = 0
    for i, (src, dst) in enumerate(pairs):
        if not (src.is_contiguous() and dst.is_contiguous()) or src.dtype != dst.dtype:
            raise ValueError("gather_rows: fields must be contiguous and of matching dtype")
        if dst.shape[0] != count or src.shape[1:] != dst.shape[1:]:
            raise ValueError("gather_rows: shape mismatch")
        row_bytes = dst[0].numel() * dst.element_size() if dst.dim() > 1 else dst.element_size()
        arr[i] = _lib.GatherField(src.data_ptr(), dst.data_ptr(), row_bytes)
        moved += 2 * row_bytes * count
    dev = indices.device
    with timer.span("gather_rows", dev, moved + 4 * count):
        rc = _lib.lib().rslrl_gather_rows(arr, len(pairs), _ptr(indices), count, ctypes.c_void_p(_stream(dev)))
    _lib.check(rc, "rslrl_gather_rows")


def gather_records(records: torch.Tensor, fields, indices: torch.Tensor):
    """Mini-batch gather over transition records (include/rslrl_amd.h rslrl_gather_records).

    records: [..., R] contiguous fp32 (one record of R floats per env-step, R % 4 == 0); fields: list of
    (offset, width, dst [count, width] contiguous fp32); dst[r] = records.view(-1, R)[indices[r], offset:offset+width].
    """
    if len(fields) > _lib.MAX_GATHER_FIELDS:
        raise ValueError(f"gather_records: at most {_lib.MAX_GATHER_FIELDS} fields per launch")
    _require_device(records, indices, *[f[2] for f in fields])
    if records.dtype != torch.float32 or not records.is_contiguous():
        raise ValueError("gather_records: records must be contiguous fp32")
    if indices.dtype != torch.int32 or not indices.is_contiguous():
        raise ValueError("gather_records: indices must be contiguous int32")
    R = records.shape[-1]
    count = indices.numel()
    arr = (_lib.RecordField * max(len(fields), 1))()
    used, moved = 0, 0
    for i, (off, width, dst) in enumerate(fields):
        if dst.dtype != torch.float32 or not dst.is_contiguous() or dst.numel() != count * width:
            raise ValueError("gather_records: dst must be contiguous fp32 [count, width]")
        arr[i] = _lib.RecordField(int(off), int(width), dst.data_ptr())
        used = max(used, off + width)
        moved += 8 * width * count
    dev = indices.device
    with timer.span("gather_rows", dev, moved + 4 * count):
        rc = _lib.lib().rslrl_gather_records(_ptr(records), R, arr, len(fields), _ptr(indices), count,
                                             ctypes.c_void_p(_stream(dev)))
    _lib.check(rc, "rslrl_gather_records")


def gather_records_side(records: torch.Tensor, fields, side: torch.Tensor, side_fields, indices: torch.Tensor):
    """gather_records plus fields of a side array (include/rslrl_amd.h rslrl_gather_records_side): side [..., 4]
    contiguous fp32 (one 16-byte unit per record index); side_fields: (offset, width, dst) with offset + width <= 4,
    dst[r] = side.view(-1, 4)[indices[r], offset:offset+width]."""
    if len(fields) + len(side_fields) > _lib.MAX_GATHER_FIELDS:
        raise ValueError(f"gather_records_side: at most {_lib.MAX_GATHER_FIELDS} fields per launch")
    _require_device(records, side, indices, *[f[2] for f in fields], *[f[2] for f in side_fields])
    if records.dtype != torch.float32 or not records.is_contiguous():
        raise ValueError("gather_records_side: records must be contiguous fp32")
    if side.dtype != torch.float32 or not side.is_contiguous() or side.shape[-1] != 4 or \
            side.numel() // 4 != records.numel() // records.shape[-1]:
        raise ValueError("gather_records_side: side must be contiguous fp32 [..., 4], one row per record")
    if indices.dtype != torch.int32 or not indices.is_contiguous():
        raise ValueError("gather_records_side: indices must be contiguous int32")
    R = records.shape[-1]
    count = indices.numel()
    arrs, moved = [], 0
    for fl in (fields, side_fields):
        arr = (_lib.RecordField * max(len(fl), 1))()
        for i, (off, width, dst) in enumerate(fl):
            if dst.dtype != torch.float32 or not dst.is_contiguous() or dst.numel() != count * width:
                raise ValueError("gather_records_side: dst must be contiguous fp32 [count, width]")
            arr[i] = _lib.RecordField(int(off), int(width), dst.data_ptr())
            moved += 8 * width * count
        arrs.append(arr)
    dev = indices.device
    with timer.span("gather_rows", dev, moved + 4 * count):
        rc = _lib.lib().rslrl_gather_records_side(_ptr(records), R, arrs[0], len(fields), _ptr(side), arrs[1],
                                                  len(side_fields), _ptr(indices), count, ctypes.c_void_p(_stream(dev)))
    _lib.check(rc, "rslrl_gather_records_side")


def record_fill_slot(records: torch.Tensor, offset: int, slot_floats: int, row=None, columns=()):
    """records.view(-1, R)[:, offset:offset + slot_floats] = [row | columns... | zeros] per record
    (include/rslrl_amd.h rslrl_record_fill_slot): row [.., w] and up to 4 columns [..] contiguous fp32, one
    entry per record."""
    _require_device(records, row, *columns)
    if records.dtype != torch.float32 or not records.is_contiguous():
        raise ValueError("record_fill_slot: records must be contiguous fp32")
    R = records.shape[-1]
    n = records.numel() // R
    rw = 0 if row is None else row.shape[-1]
    for t in ([row] if row is not None else []) + list(columns):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("record_fill_slot: row and columns must be contiguous fp32")
    if (row is not None and row.numel() != n * rw) or any(c.numel() != n for c in columns) or len(columns) > 4:
        raise ValueError("record_fill_slot: one row / value per record, at most 4 columns")
    ptrs = (ctypes.c_void_p * 4)(*[c.data_ptr() for c in columns])
    with timer.span("record_fill_slot", records.device, (4 * rw + 4 * len(columns) + 4 * slot_floats) * n):
        rc = _lib.lib().rslrl_record_fill_slot(_ptr(records), R, int(offset), int(slot_floats), _ptr(row), rw, ptrs,
                                               len(columns), n, ctypes.c_void_p(_stream(records.device)))
    _lib.check(rc, "rslrl_record_fill_slot")


# ------------------------------------------------------------------------------------------------
# ppo.py:221-315 + backward of :368
# ------------------------------------------------------------------------------------------------
STATS_LOSS, STATS_SURROGATE, STATS_VALUE, STATS_ENTROPY, STATS_KL, STATS_ADV_MEAN, STATS_ADV_STD = range(7)


def _row_stride(t: torch.Tensor, A: int) -> int:
    if t.dim() != 2 or t.shape[1] != A or t.stride(1) != 1:
        raise ValueError("ppo_loss: [B, A] operands need unit stride along actions")
    return t.stride(0)


def ppo_loss_fwd_bwd(mu, sigma, values, actions, old_logp, advantages, target_values, returns, old_mu, old_sigma, *,
                     clip_param=0.2, value_loss_coef=1.0, entropy_coef=0.01, use_clipped_value_loss=True,
                     compute_kl=True, normalize_advantage=False, grad_mu=None, grad_sigma=None, grad_values=None,
                     stats=None):
    """One fused launch sequence: loss scalars + d(loss)/d(mu, sigma, V).

    mu [B, A]; sigma [A] (shared, e.g. ActorCritic.std) or [B, A] (state-dependent std); values [B] or
    [B, 1]; actions/old_mu/old_sigma [B, A] contiguous; old_logp/advantages/target_values/returns [B]/[B, 1].
    Returns (stats[8], grad_mu [B, A], grad_sigma (shape of sigma), grad_values (shape of values)).
    """
    mu_d, sg_d, v_d = mu.detach(), sigma.detach(), values.detach()
    _require_device(mu_d, sg_d, v_d, actions, old_logp, advantages, target_values, returns, old_mu, old_sigma)
    B, A = mu_d.shape
    if A > _lib.PPO_LOSS_MAX_ACTIONS:
        raise ValueError(f"ppo_loss: at most {_lib.PPO_LOSS_MAX_ACTIONS} actions supported")
    sigma_mode = 0 if sg_d.dim() == 1 else 1
    if sigma_mode == 0 and (sg_d.numel() != A or not sg_d.is_contiguous()):
        raise ValueError("ppo_loss: shared sigma must be a contiguous [A] tensor")
    for t in (v_d, old_logp, advantages, target_values, returns):
        if t.numel() != B or not t.is_contiguous():
            raise ValueError("ppo_loss: [B] operands must be contiguous with B elements")
    gv_stride = 1
    if grad_values is not None:  # [B] / [B, 1] contiguous, or a [B, 1] column of a wider buffer
        if grad_values.numel() != B or (grad_values.dim() == 2 and grad_values.shape[1] != 1) or grad_values.dim() > 2:
            raise ValueError("ppo_loss: grad_values must hold B values ([B] or [B, 1])")
        gv_stride = grad_values.stride(0) if grad_values.dim() == 2 else (1 if grad_values.is_contiguous() else 0)
        if gv_stride < 1:
            raise ValueError("ppo_loss: grad_values rows must be evenly spaced")
    for t in (actions, old_mu, old_sigma):
        if tuple(t.shape) != (B, A) or not t.is_contiguous():
            raise ValueError("ppo_loss: actions/old_mu/old_sigma must be contiguous [B, A]")
    dev = mu_d.device
    if grad_mu is None:
        grad_mu = torch.empty((B, A), dtype=torch.float32, device=dev)
    if grad_sigma is None:
        grad_sigma = torch.empty(sg_d.shape, dtype=torch.float32, device=dev)
    if grad_values is None:
        grad_values = torch.empty(v_d.shape, dtype=torch.float32, device=dev)
    if stats is None:
        stats = torch.empty(8, dtype=torch.float32, device=dev)
    args = _lib.PPOLossArgs()
    args.B, args.A, args.sigma_mode = B, A, sigma_mode
    args.mu, args.mu_stride = mu_d.data_ptr(), _row_stride(mu_d, A)
    args.sigma = sg_d.data_ptr()
    args.sigma_stride = _row_stride(sg_d, A) if sigma_mode == 1 else 0
    args.values = v_d.data_ptr()
    args.actions, args.old_logp, args.advantages = actions.data_ptr(), old_logp.data_ptr(), advantages.data_ptr()
    args.target_values, args.returns = target_values.data_ptr(), returns.data_ptr()
    args.old_mu, args.old_sigma = old_mu.data_ptr(), old_sigma.data_ptr()
    args.clip_param, args.value_loss_coef, args.entropy_coef = clip_param, value_loss_coef, entropy_coef
    args.use_clipped_value_loss = 1 if use_clipped_value_loss else 0
    args.compute_kl = 1 if compute_kl else 0
    args.normalize_advantage = 1 if normalize_advantage else 0
    args.grad_mu, args.grad_mu_stride = grad_mu.data_ptr(), _row_stride(grad_mu, A)
    args.grad_sigma = grad_sigma.data_ptr()
    args.grad_sigma_stride = _row_stride(grad_sigma, A) if sigma_mode == 1 else 0
    args.grad_values = grad_values.data_ptr()
    args.grad_values_stride = gv_stride
    args.stats = stats.data_ptr()
    L = _lib.lib()
    ws = _ws.get(dev, "ppo_loss", L.rslrl_ppo_loss_workspace_bytes(B, A))
    # algorithmic bytes: read mu, actions, old_mu, old_sigma (+ per-row sigma) and 5 scalars per row;
    # write d mu, d V (+ per-row d sigma)
    row_bytes = 4 * (4 * A + 5) + 4 * (A + 1) + (8 * A if sigma_mode == 1 else 0)
    with timer.span("ppo_loss", dev, row_bytes * B):
        rc = L.rslrl_ppo_loss_fwd_bwd(ctypes.byref(args), _ptr(ws), ws.numel(), ctypes.c_void_p(_stream(dev)))
    _lib.check(rc, "rslrl_ppo_loss_fwd_bwd")
    return stats, grad_mu, grad_sigma, grad_values


class PPOLossFunction(torch.autograd.Function):
    """Autograd wrapper: loss = PPOLossFunction.apply(mu, sigma, values, batch..., hyper) -> scalar.

    Forward runs the fused kernel (it also produces the gradients); backward scales them by the
    upstream gradient.  The second output is the stats vector (no gradient).
    """

    @staticmethod
    def forward(ctx, mu, sigma, values, actions, old_logp, advantages, target_values, returns, old_mu, old_sigma,
                clip_param, value_loss_coef, entropy_coef, use_clipped_value_loss, compute_kl, normalize_advantage):
        stats, gmu, gsig, gv = ppo_loss_fwd_bwd(
            mu, sigma, values, actions, old_logp, advantages, target_values, returns, old_mu, old_sigma,
            clip_param=clip_param, value_loss_coef=value_loss_coef, entropy_coef=entropy_coef,
            use_clipped_value_loss=use_clipped_value_loss, compute_kl=compute_kl,
            normalize_advantage=normalize_advantage)
        ctx.save_for_backward(gmu, gsig, gv)
        ctx.mark_non_differentiable(stats)
        return stats[STATS_LOSS], stats

    @staticmethod
    def backward(ctx, g_loss, g_stats):
        gmu, gsig, gv = ctx.saved_tensors
        return (gmu * g_loss, gsig * g_loss, gv * g_loss) + (None,) * 13


# --------------------------------------------------------------------------------------------------
# rollout-side record (include/rslrl_amd.h rslrl_rollout_record)
# --------------------------------------------------------------------------------------------------
_DTYPE_CODES = {torch.float32: _lib.DTYPE_F32, torch.uint8: _lib.DTYPE_U8, torch.bool: _lib.DTYPE_U8,
                torch.int32: _lib.DTYPE_I32, torch.int64: _lib.DTYPE_I64}


def _flag_array(t, n):
    """(tensor, dtype code) for a [N] / [N, 1] flag array, converted only if its dtype is not native."""
    t = t.reshape(n)
    if t.dtype not in _DTYPE_CODES:
        t = t.float()
    if not t.is_contiguous():
        t = t.contiguous()
    return t, _DTYPE_CODES[t.dtype]


def pack_rnd_net(mlp) -> torch.Tensor:
    """[W1 | b1 | W2 | b2] of a Linear-ELU-Linear MLP (the layout rslrl_rollout_record reads)."""
    lin = [m for m in mlp if isinstance(m, torch.nn.Linear)]
    return torch.cat([lin[0].weight.reshape(-1), lin[0].bias, lin[1].weight.reshape(-1), lin[1].bias]).detach()


def rollout_record(step, *, obs_pairs, actions, mu, sigma, values, rewards, dones, time_outs, gamma,
                   out_actions, out_rewards, out_dones, out_values, out_logp, out_mu, out_sigma,
                   extra_reward=None, rnd=None, intrinsic_out=None, out_records=None):
    """One launch for the transition of env step `step` (ppo.py:142-169 + rollout_storage.py:77-103).

    obs_pairs: [(src [N, d], dst [N, d]), ...] observation groups to store.  out_records [N, R]: the obs, actions,
    mu and sigma destinations are fields of these transition records (written whole, zeros elsewhere).  rnd: None or a dict with
    keys obs [N, in], target / predictor (packed, pack_rnd_net), hidden, out, weight, and optionally
    state_mean / state_std / state_eps.  Returns nothing; all outputs are written in place."""
    _require_device(actions, mu, values, rewards)
    N, A = actions.shape
    L = _lib.lib()
    a = _lib.RolloutArgs()
    a.N, a.A = N, A
    sigma = sigma.detach()
    a.sigma_mode = 1 if sigma.dim() == 2 else 0
    keep = []

    def c(t):
        t = t.detach()
        t = t if t.is_contiguous() else t.contiguous()
        keep.append(t)
        return t.data_ptr()

    a.actions, a.mu, a.sigma, a.values, a.rewards = c(actions), c(mu), c(sigma), c(values), c(rewards.reshape(N))
    d, a.dones_dtype = _flag_array(dones, N)
    keep.append(d)
    a.dones = d.data_ptr()
    if time_outs is not None:
        to, a.time_outs_dtype = _flag_array(time_outs, N)
        keep.append(to)
        a.time_outs = to.data_ptr()
    a.gamma = float(gamma)
    if extra_reward is not None:
        a.extra_reward = c(extra_reward.reshape(N))
    if rnd is not None:
        ro = rnd["obs"]
        if ro.stride(-1) != 1:
            ro = ro.contiguous()
        keep.append(ro)
        a.rnd_obs, a.rnd_obs_stride = ro.data_ptr(), ro.stride(0)
        a.rnd_in, a.rnd_hidden, a.rnd_out = ro.shape[1], rnd["hidden"], rnd["out"]
        a.rnd_target, a.rnd_predictor = c(rnd["target"]), c(rnd["predictor"])
        a.rnd_weight = float(rnd["weight"])
        if rnd.get("state_mean") is not None:
            a.rnd_state_mean = c(rnd["state_mean"].reshape(-1))
            a.rnd_state_std = c(rnd["state_std"].reshape(-1))
            a.rnd_state_eps = float(rnd["state_eps"])
        if intrinsic_out is not None:
            a.intrinsic_out = intrinsic_out.data_ptr()
    if len(obs_pairs) > _lib.ROLLOUT_MAX_OBS:
        raise ValueError(f"at most {_lib.ROLLOUT_MAX_OBS} observation groups")
    a.n_obs = len(obs_pairs)
    for i, (src, dst) in enumerate(obs_pairs):
        a.obs[i].src, a.obs[i].dst, a.obs[i].row_floats = c(src), dst.data_ptr(), src.shape[-1]
    a.out_actions, a.out_rewards, a.out_dones = out_actions.data_ptr(), out_rewards.data_ptr(), out_dones.data_ptr()
    a.out_values, a.out_logp = out_values.data_ptr(), out_logp.data_ptr()
    a.out_mu, a.out_sigma = out_mu.data_ptr(), out_sigma.data_ptr()
    if out_records is not None:
        if out_records.dim() != 2 or out_records.shape[0] != N or not out_records.is_contiguous():
            raise ValueError("rollout_record: out_records must be contiguous [N, R]")
        a.record_floats, a.out_records = out_records.shape[1], out_records.data_ptr()
    # algorithmic bytes per env (SURVEY §8d style): obs groups in+out, actions/mu in+out, sigma out (+in if
    # per row), values/rewards/dones/time-outs in, reward/value/log-prob/done out
    obs_b = sum(8 * src.shape[-1] for src, _ in obs_pairs)
    per_env = obs_b + 4 * A * (5 + a.sigma_mode) + 4 + 4 + d.element_size() + 4 + (4 if time_outs is not None else 0) + 13
    with timer.span("rollout_record", actions.device, per_env * N):
        rc = L.rslrl_rollout_record(ctypes.byref(a), _stream(actions.device))
    _lib.check(rc, "rslrl_rollout_record")
    return keep  # the caller may hold these until the stream has consumed them (torch's allocator is stream-ordered)


class RolloutRecordPlan:
    """rollout_record's launch arguments for one storage (record layout, no RND / extra reward): the output bases, row
    strides and static fields are set once, and a step only writes its input pointers and its rows' addresses into the
    cached argument struct (rollout_record builds and checks everything per call: ~30 us of host time per env step at
    16384 envs, where the rollout is launch-bound).  `matches` tells whether a step's inputs fit the plan; the caller
    takes rollout_record otherwise."""

    _OUTS = ("out_actions", "out_rewards", "out_dones", "out_values", "out_logp", "out_mu", "out_sigma", "out_records")

    def __init__(self, outs: dict, obs_dsts, obs_widths, N: int, A: int, gamma: float, dones_dtype, time_outs_dtype,
                 shared_sigma: bool, device):
        a = _lib.RolloutArgs()
        a.N, a.A, a.sigma_mode, a.gamma = N, A, 0 if shared_sigma else 1, float(gamma)
        a.dones_dtype = _DTYPE_CODES[dones_dtype]
        self.time_outs_dtype = time_outs_dtype
        if time_outs_dtype is not None:
            a.time_outs_dtype = _DTYPE_CODES[time_outs_dtype]
        a.n_obs = len(obs_dsts)
        for i, w in enumerate(obs_widths):
            a.obs[i].row_floats = w
        rec = outs["out_records"]
        a.record_floats = rec.shape[-1]
        # [T, N, ...] buffers: row t of field f at base_f + t * stride_f (bytes)
        self.rows = [(k, outs[k].data_ptr(), outs[k].stride(0) * outs[k].element_size()) for k in self._OUTS]
        self.obs_rows = [(d.data_ptr(), d.stride(0) * d.element_size()) for d in obs_dsts]
        self.a, self.N, self.A, self.device, self.gamma = a, N, A, device, float(gamma)  # (a.gamma reads back as fp32)
        self._fn = _lib.lib().rslrl_rollout_record  # bound once: the launch runs every env step
        self.dones_dtype, self.shared_sigma, self.obs_widths = dones_dtype, shared_sigma, tuple(obs_widths)
        self.key = (self.obs_widths, dones_dtype, time_outs_dtype, self.gamma, shared_sigma)
        obs_b = sum(8 * w for w in obs_widths)
        self.bytes = (obs_b + 4 * A * (5 + (0 if shared_sigma else 1)) + 4 + 4 + torch.tensor([], dtype=dones_dtype)
                      .element_size() + 4 + (4 if time_outs_dtype is not None else 0) + 13) * N

    @staticmethod
    def signature(sigma, dones, time_outs, obs_srcs, gamma):
        """What a plan is built for (its static fields): steps with another signature need another plan."""
        return (tuple(s.shape[-1] for s in obs_srcs), dones.dtype, None if time_outs is None else time_outs.dtype,
                float(gamma), sigma.dim() == 1)

    def fits(self, actions, mu, sigma, values, rewards, dones, time_outs, obs_srcs) -> bool:
        """This step's inputs can be passed by pointer: every array dense with the element count the kernel reads
        (the general path reshapes / copies what is not), the [N, A] rows and the observation rows 16-byte aligned."""
        N, A = self.N, self.A
        for t, n in ((actions, N * A), (mu, N * A), (values, N), (rewards, N), (dones, N)):
            if t.numel() != n or not t.is_contiguous() or t.data_ptr() % 16 and n == N * A:
                return False
        if time_outs is not None and (time_outs.numel() != N or not time_outs.is_contiguous()):
            return False
        if sigma.numel() != (A if self.shared_sigma else N * A) or not sigma.is_contiguous():
            return False
        return all(s.dtype == torch.float32 and s.dim() == 2 and s.shape[0] == N and s.is_contiguous()
                   and s.data_ptr() % 16 == 0 for s in obs_srcs)

    def matches(self, actions, mu, sigma, values, rewards, dones, time_outs, obs_srcs, gamma) -> bool:
        return (self.signature(sigma, dones, time_outs, obs_srcs, gamma) == self.key
                and self.fits(actions, mu, sigma, values, rewards, dones, time_outs, obs_srcs))

    def launch(self, t: int, actions, mu, sigma, values, rewards, dones, time_outs, obs_srcs):
        a = self.a
        a.actions, a.mu, a.sigma = actions.data_ptr(), mu.data_ptr(), sigma.data_ptr()
        a.values, a.rewards, a.dones = values.data_ptr(), rewards.data_ptr(), dones.data_ptr()
        if time_outs is not None:
            a.time_outs = time_outs.data_ptr()
        for k, base, st in self.rows:
            setattr(a, k, base + t * st)
        for i, (src, (base, st)) in enumerate(zip(obs_srcs, self.obs_rows)):
            a.obs[i].src, a.obs[i].dst = src.data_ptr(), base + t * st
        with timer.span("rollout_record", self.device, self.bytes):
            rc = self._fn(ctypes.byref(a), _stream(self.device))  # the caller's current stream
        _lib.check(rc, "rslrl_rollout_record")


def ppo_tail_args(stats, kl, lr, lr32, desired_kl, sums, round_fp32=False) -> _lib.PpoTail:
    """rslrl_ppo_tail_t of the per-mini-batch tail (ppo_update_tail's arguments)."""
    _require_device(stats, kl, lr, lr32, sums)
    on = lr is not None
    return _lib.PpoTail(stats.data_ptr(), kl.data_ptr() if on else None, lr.data_ptr() if on else None,
                        lr32.data_ptr() if on else None, 1 if round_fp32 else 0,
                        float(desired_kl) * 2.0 if on else 0.0, float(desired_kl) / 2.0 if on else 0.0,
                        sums.data_ptr() if sums is not None else None)


def ppo_update_tail_args(t: _lib.PpoTail, device) -> None:
    """rslrl_ppo_update_tail of a ppo_tail_args struct (its own launch)."""
    rc = _lib.lib().rslrl_ppo_update_tail(t.stats, t.kl, t.lr, t.lr32, t.round_fp32, t.kl_hi, t.kl_lo, t.sums,
                                          _stream(device))
    _lib.check(rc, "rslrl_ppo_update_tail")


def ppo_update_tail(stats, kl, lr, lr32, desired_kl, sums, round_fp32=False):
    """One launch for the per-mini-batch tail of PPO.update (include/rslrl_amd.h rslrl_ppo_update_tail):
    the adaptive-KL lr rule on the fp64 device lr (when lr is not None; kl: fp32 device scalar) and the loss
    statistics accumulation sums[0:3] += (value, surrogate, entropy) of stats.  FusedClipAdam.step(tail=...) runs
    the same inside its norm launch."""
    ppo_update_tail_args(ppo_tail_args(stats, kl, lr, lr32, desired_kl, sums, round_fp32), stats.device)


class FusedClipAdam:
    """optimizer.step() for a torch.optim.Adam over ROCm parameters as two launches (include/rslrl_amd.h
    rslrl_clip_adam_step): gradient-norm clipping at max_grad_norm (ppo.py:373, clip_grad_norm_) folded into
    torch's fused-Adam arithmetic (ppo.py:374).  The optimizer's state (step / exp_avg / exp_avg_sq, torch's
    fused layout) and state_dict stay torch's; parameters whose grad is None are skipped, as torch does.
    Supported: one group of contiguous fp32 device parameters (at most ADAM_MAX_TENSORS), weight_decay 0,
    no amsgrad / maximize / differentiable; anything else keeps torch's clip_grad_norm_ + step."""

    def __init__(self, optimizer, max_grad_norm):
        self.opt = optimizer
        self.max_grad_norm = float(max_grad_norm) if max_grad_norm is not None else 0.0
        L = _lib.lib()
        dev = optimizer.param_groups[0]["params"][0].device
        self.ws = torch.zeros(max(L.rslrl_adam_workspace_bytes() // 4, 1), dtype=torch.int32, device=dev)
        self.args = _lib.AdamArgs()

    @staticmethod
    def supported(optimizer) -> bool:
        if not isinstance(optimizer, torch.optim.Adam) or len(optimizer.param_groups) != 1:
            return False  # the clip norm spans every gradient: one launch pair over one group
        if len(optimizer.param_groups[0]["params"]) > _lib.ADAM_MAX_TENSORS:
            return False
        for g in optimizer.param_groups:
            if g["weight_decay"] != 0 or g["amsgrad"] or g["maximize"] or g.get("differentiable", False):
                return False
            if not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in g["params"]):
                return False
        return True

    def _state(self, p):
        st = self.opt.state[p]
        if len(st) == 0:  # torch's lazy init for fused Adam (optim/adam.py _init_group)
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            return st
        # a state_dict saved by a plain (non-fused) Adam -- e.g. a reference checkpoint -- loads its step as a
        # CPU tensor (torch keeps non-fused steps on the host); the kernels read and increment it on the device
        step = st["step"]
        if not (isinstance(step, torch.Tensor) and step.device == p.device and step.dtype == torch.float32
                and step.dim() == 0):
            st["step"] = torch.tensor(float(step), dtype=torch.float32, device=p.device)
        for k in ("exp_avg", "exp_avg_sq"):
            v = st[k]
            if v.device != p.device or v.dtype != p.dtype or not v.is_contiguous():
                st[k] = v.to(device=p.device, dtype=p.dtype).contiguous()
        return st

    def adopt_loaded_state(self):
        """After optimizer.load_state_dict of a checkpoint written by a non-fused Adam: the loaded param group
        carries fused=None and CPU steps.  Re-mark the group fused (torch's fallback step then takes the tensor
        lr of update()) and move every step to its parameter's device as fp32."""
        for g in self.opt.param_groups:
            g["fused"] = True
            g["foreach"] = None
            for p in g["params"]:
                if self.opt.state.get(p):
                    self._state(p)

    def step(self, closure=None, tail=None):
        """tail: an rslrl_ppo_tail_t (ppo_tail_args) run inside the norm launch before the step sizes take the lr
        (rslrl_clip_adam_step_tail: one launch less per mini-batch than ppo_update_tail + step)."""
        if closure is not None:
            raise RuntimeError("FusedClipAdam.step: closures are not supported")
        L = _lib.lib()
        keep = []  # contiguous copies (if any) stay alive until the launch is queued
        back = []  # (grad, copy): the kernel writes the clipped gradient into the copy; .grad gets it back
        for g in self.opt.param_groups:
            chunk = [p for p in g["params"] if p.grad is not None]
            if chunk:
                a = self.args
                a.n = len(chunk)
                a.max_grad_norm = self.max_grad_norm
                lr = g["lr"]
                if isinstance(lr, torch.Tensor):
                    a.lr_dev = lr.data_ptr() if lr.is_cuda and lr.dtype == torch.float32 else None
                    a.lr = float(lr) if a.lr_dev is None else 0.0
                else:
                    a.lr_dev = None
                    a.lr = float(lr)
                a.beta1, a.beta2 = float(g["betas"][0]), float(g["betas"][1])
                a.eps = float(g["eps"])
                for i, p in enumerate(chunk):
                    st = self._state(p)
                    grad = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    keep.append(grad)
                    if grad is not p.grad:
                        back.append((p.grad, grad))
                    t = a.t[i]
                    t.param, t.grad = p.data_ptr(), grad.data_ptr()
                    t.exp_avg, t.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                    t.step, t.numel = st["step"].data_ptr(), p.numel()
                if tail is not None:
                    rc = L.rslrl_clip_adam_step_tail(ctypes.byref(a), ctypes.byref(tail), self.ws.data_ptr(),
                                                     self.ws.numel() * 4, _stream(self.ws.device))
                    tail = None
                else:
                    rc = L.rslrl_clip_adam_step(ctypes.byref(a), self.ws.data_ptr(), self.ws.numel() * 4,
                                                _stream(self.ws.device))
                _lib.check(rc, "rslrl_clip_adam_step")
        if tail is not None:  # no group had gradients: the tail still runs
            ppo_update_tail_args(tail, self.ws.device)
        for g, c in back:
            g.copy_(c)
        return None



# --------------------------------------------------------------------------------------------------
# ppo.py:352-363 + :369-372 -- RND predictor loss and gradient of one mini-batch
# --------------------------------------------------------------------------------------------------
def rnd_linears(mlp):
    """(Linear, Linear) of a Linear-ELU(alpha 1)-Linear MLP whose sizes the fused RND kernels take, else None."""
    mods = list(mlp)
    lin = [m for m in mods if isinstance(m, torch.nn.Linear)]
    if (len(mods) != 3 or len(lin) != 2 or not isinstance(mods[1], torch.nn.ELU) or mods[1].alpha != 1.0
            or lin[0].in_features > _lib.RND_MAX_IN or lin[0].out_features > _lib.RND_MAX_HIDDEN
            or lin[1].out_features > _lib.RND_MAX_OUT or lin[1].in_features != lin[0].out_features):
        return None
    if any(not (t.is_contiguous() and t.dtype == torch.float32) for m in lin for t in (m.weight, m.bias)):
        return None
    return lin[0], lin[1]


def rnd_update(state, predictor, target, target_embedding, grad, loss_sum=None, loss=None, state_mean=None,
               state_std=None, state_eps=0.0):
    """One launch pair for the RND predictor's training step of a mini-batch (include/rslrl_amd.h rslrl_rnd_update).

    state [B, in] fp32 (unit column stride); predictor / target: (Linear, Linear) of rnd_linears; target None:
    target_embedding [B, out] holds the (detached) target values already, else they are computed and, when
    target_embedding is given, stored there.  grad: contiguous fp32 of the predictor's parameter count, packed
    [dW1 | db1 | dW2 | db2] -- overwritten.  loss_sum (fp64 [1], optional) += the fp32 mse; loss (fp32 [1]) = mse."""
    l1, l2 = predictor
    B, n_in = state.shape
    H, Q = l1.out_features, l2.out_features
    _require_device(state, grad, target_embedding, loss_sum, loss, state_mean, state_std)
    if state.dtype != torch.float32 or state.stride(1) != 1:
        raise ValueError("rnd_update: state must be fp32 with unit column stride")
    if n_in != l1.in_features:
        raise ValueError(f"rnd_update: state has {n_in} columns, the predictor takes {l1.in_features}")
    P = H * n_in + H + Q * H + Q
    if grad.dtype != torch.float32 or not grad.is_contiguous() or grad.numel() != P:
        raise ValueError("rnd_update: grad must be a contiguous fp32 buffer of the predictor's parameter count")
    if target_embedding is not None and (target_embedding.dtype != torch.float32 or not target_embedding.is_contiguous()
                                         or target_embedding.numel() != B * Q):
        raise ValueError("rnd_update: target_embedding must be contiguous fp32 [B, out]")
    a = _lib.RndUpdateArgs()
    a.B, a.in_, a.hidden, a.out = B, n_in, H, Q
    a.state, a.state_stride = state.data_ptr(), state.stride(0)
    if state_mean is not None:
        a.state_mean, a.state_std, a.state_eps = state_mean.data_ptr(), state_std.data_ptr(), float(state_eps)
    a.pred_w1, a.pred_b1 = l1.weight.data_ptr(), l1.bias.data_ptr()
    a.pred_w2, a.pred_b2 = l2.weight.data_ptr(), l2.bias.data_ptr()
    if target is not None:
        t1, t2 = target
        if (t1.in_features, t1.out_features, t2.out_features) != (n_in, H, Q):
            raise ValueError("rnd_update: predictor and target must have the same shapes")
        a.target_w1, a.target_b1 = t1.weight.data_ptr(), t1.bias.data_ptr()
        a.target_w2, a.target_b2 = t2.weight.data_ptr(), t2.bias.data_ptr()
    elif target_embedding is None:
        raise ValueError("rnd_update: without the target network the target embedding must be given")
    a.target_embedding = target_embedding.data_ptr() if target_embedding is not None else None
    a.grad = grad.data_ptr()
    a.loss_sum = loss_sum.data_ptr() if loss_sum is not None else None
    a.loss = loss.data_ptr() if loss is not None else None
    L = _lib.lib()
    dev = state.device
    ws = _ws.get(dev, "rnd", L.rslrl_rnd_update_workspace_bytes(B, n_in, H, Q))
    with timer.span("rnd_update", dev, 4 * (n_in + Q) * B, 2 * B * (3 if target is not None else 2) * (H * n_in + Q * H)):
        rc = L.rslrl_rnd_update(ctypes.byref(a), _ptr(ws), ws.numel(), ctypes.c_void_p(_stream(dev)))
    _lib.check(rc, "rslrl_rnd_update")
