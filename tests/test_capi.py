"""The C ABI library loads, exports every entry point include/rslrl_amd.h declares, and validates its
arguments before touching the GPU (no compute calls here: this runs without a GPU)."""

import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, golden_path
from rsl_rl_amd import _lib

HEADER = os.path.join(ROOT, "include", "rslrl_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rslrl_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding_list():
    assert declared_functions() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.rslrl_abi_version() == _lib.ABI_VERSION


def test_status_strings():
    L = _lib.lib()
    assert L.rslrl_status_string(0) == b"ok"
    assert b"invalid" in L.rslrl_status_string(-1)
    assert b"hipError_t" in L.rslrl_status_string(1)


def test_argument_validation_without_gpu():
    L = _lib.lib()
    # negative sizes / null pointers are rejected before any launch
    assert L.rslrl_compute_returns(None, None, None, None, 0.99, 0.95, -1, 4, 1, None, None, None, 0, None) == -1
    assert L.rslrl_compute_returns(None, None, None, None, 0.99, 0.95, 4, 4, 1, None, None, None, 0, None) == -1
    assert L.rslrl_compute_returns(None, None, None, None, 0.99, 0.95, 0, 4, 1, None, None, None, 0, None) == 0
    f = (_lib.GatherField * 1)(_lib.GatherField(8, 8, 6))  # row_bytes not a multiple of 4
    assert L.rslrl_gather_rows(f, 1, 8, 4, None) == -1
    assert L.rslrl_gather_rows(f, 17, 8, 4, None) == -1
    args = _lib.PPOLossArgs()
    args.B, args.A = 0, 4
    assert L.rslrl_ppo_loss_fwd_bwd(ctypes.byref(args), None, 0, None) == -1
    args.B, args.A = 10, 65
    assert L.rslrl_ppo_loss_fwd_bwd(ctypes.byref(args), None, 0, None) == -1
    assert L.rslrl_ppo_loss_workspace_bytes(393216, 12) >= 8 * 16 * 512
    assert L.rslrl_compute_returns_workspace_bytes(24, 65536) >= 16 * 256


def test_gae_workspace_words_and_knobs_without_gpu():
    """ABI 18: the status word sits after the partials and the barrier's ticket / generation, inside the workspace;
    the test knobs validate their names and ranges and hand back the previous value (host code, no GPU)."""
    L = _lib.lib()
    ws = L.rslrl_compute_returns_workspace_bytes(24, 131072)
    off = L.rslrl_compute_returns_status_offset()
    assert off % 4 == 0 and off >= 8 + 2048 * 32 and off + 4 <= ws
    prev = ctypes.c_int64(0)
    assert L.rslrl_debug_knob(b"no_such_knob", 1, None) == -1
    assert L.rslrl_debug_knob(None, 1, None) == -1
    assert L.rslrl_debug_knob(b"gae_spin_limit", -1, None) == -1
    assert L.rslrl_debug_knob(b"gae_spin_limit", 5, ctypes.byref(prev)) == 0
    assert prev.value == 1 << 22
    assert L.rslrl_debug_knob(b"gae_spin_limit", prev.value, ctypes.byref(prev)) == 0 and prev.value == 5
    assert L.rslrl_debug_knob(b"gae_form", -1, ctypes.byref(prev)) == 0 and prev.value == -1
    # forms need T in {8, 16, 24, 32} for a one-launch form; invalid sizes report the two-launch form
    assert L.rslrl_compute_returns_slots_form(0, 4, None, None, None, None, None, None) == 0
    assert L.rslrl_compute_returns_slots_form(5, 4096, None, None, None, None, None, None) == 0


def test_value_head_partial_rows_follows_the_dispatch():
    """ABI 18: a call with colsum_partials always takes the tiled head, so its partial-row count is M / 128
    whatever the streaming default; without it the streaming form's per-slice count (<= 256 rows)."""
    L = _lib.lib()
    M = 393216
    assert L.rslrl_value_head_partial_rows(M, 1) == M // 128
    assert L.rslrl_value_head_partial_rows(M, 0) in (M // 128,) or L.rslrl_value_head_partial_rows(M, 0) <= 256
    assert L.rslrl_value_head_partial_rows(0, 0) == 0


def test_linear_abi_rejects_bad_shapes():
    L = _lib.lib()
    assert L.rslrl_linear_fwd(8, 10, 6, 8, 16, 8, 1, 8, None, None) == -1  # K % 4 != 0
    assert L.rslrl_linear_fwd(8, 10, 8, 8, 300, 8, 1, 8, None, None) == -1  # N > 256
    assert L.rslrl_linear_fwd(8, 0, 8, 8, 16, 8, 1, 8, None, None) == 0  # empty batch
    assert L.rslrl_linear_fwd(16, 10, 8, None, 16, 16, 1, 16, None, None) == -1  # no weight and no image
    assert L.rslrl_linear_fwd(16, 10, 8, None, 16, 16, 1, 16, 24, None) == -4  # misaligned image
    assert L.rslrl_linear_dgrad_elu(8, 10, 6, 8, 16, 8, 8, 8, None, None) == -1  # Nred % 4 != 0
    assert L.rslrl_linear_tiles(393216) == 3072
    assert L.rslrl_linear_bimage_bytes(256) == 16 * 3 * 256 * 32  # 16 chunks x 3 planes x 256 rows x 32 B
    assert L.rslrl_linear_bimage_bytes(12) == 3 * 256 * 32
    assert L.rslrl_linear_prepare_bimage(16, 300, 16, 0, 16, None) == -1  # rows > 256
    assert L.rslrl_linear_prepare_bimage(16, 16, 16, 0, 8, None) == -4  # misaligned image


def test_pair_and_optimizer_abi_validation():
    L = _lib.lib()
    a0 = _lib.LinearArgs(_lib.LINEAR_FWD_ELU, _lib.ARITH_X6, 16, None, 128, 48, 256, 16, 16, None, 16)
    a1 = _lib.LinearArgs(_lib.LINEAR_FWD_ELU, _lib.ARITH_X6, 16, None, 64, 48, 256, 16, 16, None, 16)
    assert L.rslrl_linear_gemm_pair(ctypes.byref(a0), ctypes.byref(a1), None) == -1  # different M
    a1.M, a1.op = 128, _lib.LINEAR_DGRAD_ELU
    assert L.rslrl_linear_gemm_pair(ctypes.byref(a0), ctypes.byref(a1), None) == -3  # not a forward pair
    a1.op = _lib.LINEAR_FWD_ELU
    a0.M = a1.M = 0
    assert L.rslrl_linear_gemm_pair(ctypes.byref(a0), ctypes.byref(a1), None) == 0  # empty batch: no launch
    assert L.rslrl_linear_gemm_pair(None, ctypes.byref(a1), None) == -1
    args = _lib.AdamArgs()
    ws_bytes = L.rslrl_adam_workspace_bytes()
    assert ws_bytes >= 256 + 128 * 8 + 4
    args.n = 0
    assert L.rslrl_clip_adam_step(ctypes.byref(args), 16, ws_bytes, None) == -1  # no tensors
    args.n = _lib.ADAM_MAX_TENSORS + 1
    assert L.rslrl_clip_adam_step(ctypes.byref(args), 16, ws_bytes, None) == -1  # too many tensors
    args.n = 1
    assert L.rslrl_clip_adam_step(ctypes.byref(args), 16, ws_bytes - 1, None) == -2  # workspace too small
    assert L.rslrl_clip_adam_step(ctypes.byref(args), 16, ws_bytes, None) == -1  # null tensor pointers


def test_randperm_rejects_bad_state():
    L = _lib.lib()
    out = np.empty(10, np.int32)
    bad = np.zeros(100, np.uint8)
    assert L.rslrl_randperm_mt19937(bad.ctypes.data, bad.nbytes, 10, out.ctypes.data) == -5
    st = torch.Generator().manual_seed(0).get_state().numpy().copy()
    st[8:12] = np.frombuffer(np.int32(9999).tobytes(), np.uint8)  # left out of range
    assert L.rslrl_randperm_mt19937(st.ctypes.data, st.nbytes, 10, out.ctypes.data) == -5


def test_hot_path_refuses_cpu_tensors():
    from rsl_rl_amd import kernels

    t = torch.zeros(4, 3, 1)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        kernels.compute_returns(t, t, t.to(torch.uint8), torch.zeros(3, 1), 0.99, 0.95, True, t.clone(), t.clone())
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        kernels.normalize_advantages_(torch.zeros(8))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        kernels.gather_rows([(torch.zeros(4, 2), torch.zeros(2, 2))], torch.zeros(2, dtype=torch.int32))


def test_golden_files_present():
    for f in ("gae.npz", "perm.npz", "minibatch.npz", "update_c1.npz", "golden.json"):
        assert os.path.exists(golden_path(f)), f
