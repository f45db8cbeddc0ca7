"""HIP multi-field gather + RolloutStorage.mini_batch_generator vs the golden mini-batches and the oracle
(bit-exact: integer indices and gathered fp32 rows)."""

import numpy as np
import pytest
import torch

from conftest import golden_path
from oracle import ppo_oracle as O
from rsl_rl_amd import kernels
from rsl_rl_amd.storage import RolloutStorage, rollout_storage

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("row_elems", [1, 3, 4, 12, 48, 50, 257, 1100])
def test_gather_rows_vs_oracle(row_elems, cuda_device):
    rng = np.random.default_rng(row_elems)
    rows, count = 5000, 3001
    src = rng.standard_normal((rows, row_elems), dtype=np.float32)
    idx = rng.integers(0, rows, count).astype(np.int32)
    s = torch.from_numpy(src).to(cuda_device)
    d = torch.empty(count, row_elems, device=cuda_device)
    kernels.gather_rows([(s, d)], torch.from_numpy(idx).to(cuda_device))
    assert np.array_equal(d.cpu().numpy(), O.gather_rows(src, idx.astype(np.int64)))


def test_gather_many_fields_and_misaligned(cuda_device):
    rng = np.random.default_rng(0)
    rows, count = 777, 600
    idx = torch.from_numpy(rng.integers(0, rows, count).astype(np.int32)).to(cuda_device)
    pairs, refs = [], []
    for k in range(20):  # > RSLRL_MAX_GATHER_FIELDS -> split into several launches
        w = 1 + (k * 7) % 23
        base = torch.from_numpy(rng.standard_normal((rows * w + 1,), dtype=np.float32)).to(cuda_device)
        src = base[1:].view(rows, w) if k % 3 == 0 else base[: rows * w].view(rows, w)  # misaligned start
        dst = torch.empty(count, w, device=cuda_device)
        pairs.append((src, dst))
        refs.append(O.gather_rows(src.cpu().numpy(), idx.cpu().numpy().astype(np.int64)))
    kernels.gather_rows(pairs, idx)
    for (_, dst), ref in zip(pairs, refs):
        assert np.array_equal(dst.cpu().numpy(), ref)


def test_golden_minibatches(golden_meta, cuda_device):
    m = golden_meta["minibatch"]
    z = np.load(golden_path("minibatch.npz"))
    T, N, A = m["T"], m["N"], m["A"]
    obs0 = {"policy": torch.zeros(N, 3), "extra": torch.zeros(N, 2)}
    st = RolloutStorage("rl", N, T, obs0, [A], cuda_device)
    st.observations["policy"].copy_(torch.from_numpy(z["in/obs_policy"]))
    st.observations["extra"].copy_(torch.from_numpy(z["in/obs_extra"]))
    for k in ("actions", "values", "returns", "actions_log_prob", "advantages", "mu", "sigma"):
        getattr(st, k).copy_(torch.from_numpy(z[f"in/{k}"]))
    torch.manual_seed(m["torch_seed"])
    names = ["actions", "target_values", "advantages", "returns", "old_logp", "old_mu", "old_sigma"]
    batches = list(st.mini_batch_generator(m["M"], m["E"]))
    assert len(batches) == m["num_batches"]
    for j, b in enumerate(batches):
        assert np.array_equal(b[0]["policy"].cpu().numpy(), z[f"mb{j}/obs_policy"])
        assert np.array_equal(b[0]["extra"].cpu().numpy(), z[f"mb{j}/obs_extra"])
        for nm, t in zip(names, b[1:8]):
            assert np.array_equal(t.cpu().numpy(), z[f"mb{j}/{nm}"]), (j, nm)
        assert b[8] == (None, None) and b[9] is None


def test_permutation_contents_and_tail_drop(cuda_device):
    """N*T not divisible by M: the tail is dropped and the permutation covers range(M*mb) exactly."""
    T, N, M = 5, 37, 4
    st = RolloutStorage("rl", N, T, {"policy": torch.zeros(N, 2)}, [3], cuda_device)
    st.observations["policy"].copy_(torch.arange(T * N * 2, dtype=torch.float32).view(T, N, 2))
    g = torch.Generator().manual_seed(9)
    st.perm_generator = g
    batches = list(st.mini_batch_generator(M, 2))
    mb = (T * N) // M
    idx = st.last_indices.cpu().long()
    assert idx.numel() == M * mb and torch.equal(idx.sort().values, torch.arange(M * mb))
    ref = torch.randperm(M * mb, generator=torch.Generator().manual_seed(9))
    assert torch.equal(idx, ref)
    flat = st.observations["policy"].flatten(0, 1).cpu()
    for i, b in enumerate(batches[:M]):
        assert torch.equal(b[0]["policy"].cpu(), flat[ref[i * mb:(i + 1) * mb]])
    # epochs reuse the same permutation (rollout_storage.py:165 is outside the epoch loop)
    for i in range(M):
        assert torch.equal(batches[i][0]["policy"], batches[M + i][0]["policy"])


@pytest.mark.parametrize("M,stage", [(2, False), (1, False), (2, True)])
def test_prefetched_permutation_matches_plain_draws(M, stage, cuda_device, monkeypatch):
    """The same sequence of updates with and without interference: every permutation equals torch.randperm on
    the generator's state at that call, and the generator's state after each update matches.  The prefetch starts
    at the second mini-batch: with one mini-batch per update every draw is synchronous.  stage: the drawn-ahead
    permutation is uploaded early (stage_permutation, as compute_returns does), the reseed included."""
    T, N = 4, 50
    n = (T * N // M) * M
    st = RolloutStorage("rl", N, T, {"policy": torch.zeros(N, 2)}, [3], cuda_device)
    st.perm_generator = torch.Generator().manual_seed(21)
    ref = torch.Generator().manual_seed(21)
    staged = 0
    for k in range(6):
        if k == 3:  # reseed both between two updates: the prepared permutation is stale and must be dropped
            st.perm_generator.manual_seed(5)
            ref.manual_seed(5)
        if stage:
            monkeypatch.setattr(rollout_storage, "_STAGE_PERM", True)
            if st._prefetch is not None:
                st._prefetch[4].join()  # the worker's draw is done (the rollout takes far longer in a run)
            st.stage_permutation()
            staged += st._prefetch is not None and len(st._prefetch) == 8
        for _ in st.mini_batch_generator(M, 1):
            pass
        expect = torch.randperm(n, generator=ref)
        assert torch.equal(st.last_indices.cpu().long(), expect), k
        assert torch.equal(st.perm_generator.get_state(), ref.get_state()), k
    assert staged == (5 if stage else 0)  # every update but the first finds a drawn-ahead permutation


@pytest.mark.parametrize("R,fields", [
    (96, [(0, 48), (48, 12), (84, 1), (85, 1), (86, 1), (87, 1), (60, 12), (72, 12)]),  # C3's record
    (32, [(0, 3), (3, 5), (8, 4), (13, 1)]),  # odd widths / offsets: 4-byte path
    (160, [(0, 132), (132, 4), (136, 1), (140, 8)]),  # > 128 used floats: 32-row tiles
    (256, [(0, 256)]),  # the maximum
])
def test_gather_records_vs_oracle(R, fields, cuda_device):
    rng = np.random.default_rng(R)
    rows, count = 3000, 2777  # a ragged last tile
    src = rng.standard_normal((rows, R), dtype=np.float32)
    idx = rng.integers(0, rows, count).astype(np.int32)
    rec = torch.from_numpy(src).to(cuda_device)
    outs = [(o, w, torch.empty(count, w, device=cuda_device)) for o, w in fields]
    kernels.gather_records(rec, outs, torch.from_numpy(idx).to(cuda_device))
    for o, w, d in outs:
        ref = O.gather_rows(np.ascontiguousarray(src[:, o:o + w]), idx.astype(np.int64))
        assert np.array_equal(d.cpu().numpy(), ref), (o, w)


@pytest.mark.parametrize("offset,slot,rw,ncols", [(80, 16, 12, 4), (48, 16, 8, 4), (4, 8, 0, 3), (0, 64, 60, 4)])
def test_record_fill_slot(offset, slot, rw, ncols, cuda_device):
    rng = np.random.default_rng(offset + rw)
    T, N, R = 5, 1031, 96 if offset + slot > 64 else 64
    base = rng.standard_normal((T, N, R), dtype=np.float32)
    rec = torch.from_numpy(base).to(cuda_device)
    row = torch.from_numpy(rng.standard_normal((T, N, rw), dtype=np.float32)).to(cuda_device) if rw else None
    cols = [torch.from_numpy(rng.standard_normal((T, N, 1), dtype=np.float32)).to(cuda_device) for _ in range(ncols)]
    kernels.record_fill_slot(rec, offset, slot, row=row, columns=cols)
    ref = base.copy()
    ref[:, :, offset:offset + slot] = 0
    if rw:
        ref[:, :, offset:offset + rw] = row.cpu().numpy()
    for j, c in enumerate(cols):
        ref[:, :, offset + rw + j] = c.cpu().numpy()[:, :, 0]
    assert np.array_equal(rec.cpu().numpy(), ref)


def _fill_storage(st, rng, T, N, groups, A):
    for k, d in groups.items():
        st.observations[k].copy_(torch.from_numpy(rng.standard_normal((T, N, d), dtype=np.float32)))
    for k in ("actions", "values", "returns", "actions_log_prob", "advantages", "mu", "sigma"):
        shape = (T, N, A) if k in ("actions", "mu", "sigma") else (T, N, 1)
        getattr(st, k).copy_(torch.from_numpy(rng.standard_normal(shape, dtype=np.float32)))


def test_record_storage_minibatches_bit_exact(cuda_device, monkeypatch):
    """The record layout (two observation groups, A = 8) yields exactly the reference's
    field.flatten(0, 1)[indices[mb]] for every field, like the one-buffer-per-field layout."""
    T, N, A, M, E = 6, 333, 8, 3, 2
    groups = {"policy": 20, "critic": 12}
    obs0 = {k: torch.zeros(N, d) for k, d in groups.items()}
    st = RolloutStorage("rl", N, T, obs0, [A], cuda_device)
    assert st.records is not None and st.records.shape[-1] == 64  # 20 + 12 + 24 = 56 used floats -> 64
    monkeypatch.setenv("RSLRL_RECORD_LAYOUT", "0")
    soa = RolloutStorage("rl", N, T, obs0, [A], cuda_device)
    assert soa.records is None
    _fill_storage(st, np.random.default_rng(3), T, N, groups, A)
    _fill_storage(soa, np.random.default_rng(3), T, N, groups, A)
    st.perm_generator = torch.Generator().manual_seed(4)
    soa.perm_generator = torch.Generator().manual_seed(4)
    got = list(st.mini_batch_generator(M, E))
    ref = list(soa.mini_batch_generator(M, E))
    idx = st.last_indices.cpu().long()
    mb = (T * N) // M
    flat = {k: getattr(soa, k).flatten(0, 1).cpu() for k in ("actions", "values", "advantages", "returns",
                                                           "actions_log_prob", "mu", "sigma")}
    names = ["actions", "values", "advantages", "returns", "actions_log_prob", "mu", "sigma"]
    for j, (g, r) in enumerate(zip(got, ref)):
        sel = idx[(j % M) * mb:(j % M + 1) * mb]
        for k in groups:
            assert torch.equal(g[0][k].cpu(), r[0][k].cpu())
            assert torch.equal(g[0][k].cpu(), soa.observations[k].flatten(0, 1).cpu()[sel])
        for nm, a, b in zip(names, g[1:8], r[1:8]):
            assert torch.equal(a.cpu(), b.cpu()), (j, nm)
            assert torch.equal(a.cpu(), flat[nm][sel]), (j, nm)


@pytest.mark.parametrize("T,N", [(24, 4096), (5, 1031), (1, 3)])
def test_compute_returns_records_matches_scan_plus_slot_copy(T, N, cuda_device):
    """rslrl_compute_returns_records == rslrl_compute_returns (normalised) + rslrl_record_fill_slot, bit for bit:
    the contiguous returns / advantages and every record (the slot written whole, the rest untouched)."""
    rng = np.random.default_rng(T * N)
    R, off = 96, 88
    f = lambda *s: torch.from_numpy(rng.standard_normal(s, dtype=np.float32)).to(cuda_device)  # noqa: E731
    values, rewards, logp, last = f(T, N, 1), f(T, N, 1), f(T, N, 1), f(N, 1)
    dones = torch.from_numpy((rng.random((T, N, 1)) < 0.05).astype(np.uint8)).to(cuda_device)
    rec0 = f(T, N, R)
    ret_a, adv_a = torch.empty_like(values), torch.empty_like(values)
    ret_b, adv_b = torch.empty_like(values), torch.empty_like(values)
    rec_a, rec_b = rec0.clone(), rec0.clone()
    kernels.compute_returns(values, rewards, dones, last, 0.99, 0.95, True, ret_a, adv_a)
    kernels.record_fill_slot(rec_a, off, 8, columns=[values, logp, ret_a, adv_a])
    kernels.compute_returns_records(values, rewards, dones, last, 0.99, 0.95, ret_b, adv_b, logp, rec_b, off)
    assert torch.equal(ret_a, ret_b) and torch.equal(adv_a, adv_b)
    assert torch.equal(rec_a, rec_b)


@pytest.mark.parametrize("T,N", [(24, 4096), (5, 1031), (1, 3), (24, 65536), (8, 1031), (16, 300), (32, 131072),
                                 (24, 300000)])
def test_compute_returns_slots_matches_scan_plus_stack(T, N, cuda_device):
    """rslrl_compute_returns_slots == rslrl_compute_returns (normalised) followed by stacking {value, log-prob, return,
    advantage} per env-step, bit for bit (returns, advantages and the whole slot array).  T in {8, 16, 24, 32} with
    every block resident takes the one-launch form (scan + grid barrier + normalisation, round 5); T = 5, T = 1 and
    N = 300000 (more blocks than the partial array holds) the scan + normaliser pair: both must equal the plain path."""
    rng = np.random.default_rng(T * N + 1)
    f = lambda *s: torch.from_numpy(rng.standard_normal(s, dtype=np.float32)).to(cuda_device)  # noqa: E731
    values, rewards, logp, last = f(T, N, 1), f(T, N, 1), f(T, N, 1), f(N, 1)
    dones = torch.from_numpy((rng.random((T, N, 1)) < 0.05).astype(np.uint8)).to(cuda_device)
    ret_a, adv_a = torch.empty_like(values), torch.empty_like(values)
    ret_b, adv_b = torch.empty_like(values), torch.empty_like(values)
    slots = torch.full((T, N, 4), float("nan"), device=cuda_device)
    kernels.compute_returns(values, rewards, dones, last, 0.99, 0.95, True, ret_a, adv_a)
    kernels.compute_returns_slots(values, rewards, dones, last, 0.99, 0.95, ret_b, adv_b, logp, slots)
    assert torch.equal(ret_a, ret_b) and torch.equal(adv_a, adv_b)
    assert torch.equal(slots, torch.cat([values, logp, ret_a, adv_a], dim=-1))


def test_compute_returns_slots_one_launch_rearms(cuda_device):
    """The one-launch form's grid barrier leaves its ticket at zero and raises no error word, so back-to-back calls
    (and a call after the two-launch path used the same workspace) give the same bits."""
    T, N = 24, 65536
    rng = np.random.default_rng(7)
    f = lambda *s: torch.from_numpy(rng.standard_normal(s, dtype=np.float32)).to(cuda_device)  # noqa: E731
    values, rewards, logp, last = f(T, N, 1), f(T, N, 1), f(T, N, 1), f(N, 1)
    dones = torch.from_numpy((rng.random((T, N, 1)) < 0.05).astype(np.uint8)).to(cuda_device)
    outs = []
    for _ in range(3):
        ret, adv = torch.empty_like(values), torch.empty_like(values)
        slots = torch.full((T, N, 4), float("nan"), device=cuda_device)
        kernels.compute_returns_slots(values, rewards, dones, last, 0.99, 0.95, ret, adv, logp, slots)
        kernels.compute_returns(values, rewards, dones, last, 0.99, 0.95, True, torch.empty_like(values),
                                torch.empty_like(values))
        outs.append((ret, adv, slots))
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(outs[0], o))
    L = kernels._lib.lib()
    ws = kernels._gae_workspace(values.device, T, N)
    off = L.rslrl_compute_returns_status_offset() - 8  # [ticket][-][status]; group 0's generation 256 bytes on
    words = ws[off:off + 12].view(torch.int32).cpu().tolist()
    gen0 = ws[off + 256:off + 260].view(torch.int32).item()
    assert words[0] == 0 and words[2] == 0, words  # ticket re-armed, no barrier time-out
    assert gen0 >= 3  # the generation advanced once per one-launch call


@pytest.mark.parametrize("R,used", [(96, 84), (64, 56), (256, 252)])
def test_gather_records_side_bit_exact(R, used, cuda_device):
    """rslrl_gather_records_side: record fields and the side array's units of each drawn row, bit for bit
    (incl. a record that fills all 256 floats, misaligned scalar destinations and a ragged row count)."""
    g = torch.Generator(device=cuda_device).manual_seed(R)
    n, rows = 3 * 1031, 2 * 1031 + 5
    rec = torch.randn(n, R, device=cuda_device, generator=g)
    side = torch.randn(n, 4, device=cuda_device, generator=g)
    idx = torch.randint(0, n, (rows,), device=cuda_device, generator=g, dtype=torch.int32)
    widths = [(0, used - 24), (used - 24, 12), (used - 12, 12)]
    dst = [torch.empty(rows, w, device=cuda_device) for _, w in widths]
    big = torch.empty(rows * 4 + 1, device=cuda_device)
    sdst = [big[1 + k * rows: 1 + (k + 1) * rows].view(rows, 1) for k in range(4)]  # 4-byte aligned only
    kernels.gather_records_side(rec, [(o, w, d) for (o, w), d in zip(widths, dst)], side,
                                [(k, 1, sdst[k]) for k in range(4)], idx)
    il = idx.long()
    for (o, w), d in zip(widths, dst):
        assert torch.equal(d, rec[il, o:o + w])
    for k in range(4):
        assert torch.equal(sdst[k][:, 0], side[il, k])


def test_storage_slot_from_compute_returns_and_invalidation(cuda_device, monkeypatch):
    """The record storage's slots written by compute_returns give the same mini-batches as the per-field layout;
    an in-place write to a scalar buffer after compute_returns (or a new transition) makes the generator copy the
    slots again instead of gathering stale ones."""
    T, N, A, M = 4, 257, 8, 2
    groups = {"policy": 20}
    obs0 = {k: torch.zeros(N, d) for k, d in groups.items()}
    st = RolloutStorage("rl", N, T, obs0, [A], cuda_device)
    monkeypatch.setenv("RSLRL_RECORD_LAYOUT", "0")
    soa = RolloutStorage("rl", N, T, obs0, [A], cuda_device)
    assert st.records is not None and soa.records is None
    _fill_storage(st, np.random.default_rng(8), T, N, groups, A)
    _fill_storage(soa, np.random.default_rng(8), T, N, groups, A)
    for s in (st, s2 := soa):
        s.rewards.copy_(torch.linspace(-1, 1, T * N).view(T, N, 1))
        s.dones.zero_()
    last = torch.linspace(0, 1, N, device=cuda_device).view(N, 1)
    calls = []
    real = kernels.record_fill_slot
    monkeypatch.setattr(kernels, "record_fill_slot", lambda *a, **k: (calls.append(1), real(*a, **k))[1])

    def batches(s, seed):
        s.perm_generator = torch.Generator().manual_seed(seed)
        return [tuple(t.cpu() for t in b[1:8]) for b in s.mini_batch_generator(M, 1)]

    for s in (st, s2):
        s.compute_returns(last, 0.99, 0.95, normalize_advantage=True)
    assert all(torch.equal(a, b) for x, y in zip(batches(st, 1), batches(s2, 1)) for a, b in zip(x, y))
    assert not calls  # the slots came from compute_returns
    for s in (st, s2):
        s.returns.mul_(2.0)  # an in-place edit between compute_returns and the update
    assert all(torch.equal(a, b) for x, y in zip(batches(st, 2), batches(s2, 2)) for a, b in zip(x, y))
    assert len(calls) == 1
    assert all(torch.equal(a, b) for x, y in zip(batches(st, 3), batches(s2, 3)) for a, b in zip(x, y))
    assert len(calls) == 1  # still valid: nothing changed since the copy
