"""HIP GAE (rslrl_compute_returns) vs the golden vectors and the oracle.

Bit-exact: returns and un-normalised advantages.  Normalised advantages: |diff| <= 1e-5 * (1 + |x|)
(fp64 statistics, summation order differs from torch's fp32 mean/std).
"""

import numpy as np
import pytest
import torch

from conftest import golden_path
from oracle import ppo_oracle as O
from rsl_rl_amd import kernels

pytestmark = pytest.mark.gpu


def _run(values, rewards, dones, last_values, gamma, lam, normalize, dev):
    T, N = values.shape
    v = torch.from_numpy(values).reshape(T, N, 1).to(dev)
    r = torch.from_numpy(rewards).reshape(T, N, 1).to(dev)
    d = torch.from_numpy(dones).reshape(T, N, 1).to(dev)
    lv = torch.from_numpy(last_values).reshape(N, 1).to(dev)
    ret = torch.empty(T, N, 1, device=dev)
    adv = torch.empty(T, N, 1, device=dev)
    kernels.compute_returns(v, r, d, lv, gamma, lam, normalize, ret, adv)
    torch.cuda.synchronize()
    return ret.cpu().numpy().reshape(T, N), adv.cpu().numpy().reshape(T, N)


def test_golden(golden_meta, cuda_device):
    z = np.load(golden_path("gae.npz"))
    for name, m in sorted(golden_meta["gae"].items()):
        g = lambda k: z[f"{name}/{k}"]  # noqa: E731
        args = (g("values"), g("rewards"), g("dones"), g("last_values"), m["gamma"], m["lam"])
        ret, adv = _run(*args, False, cuda_device)
        assert np.array_equal(ret, g("returns")), name
        assert np.array_equal(adv, g("advantages_raw")), name
        ret2, advn = _run(*args, True, cuda_device)
        assert np.array_equal(ret2, g("returns")), name
        ref = g("advantages_norm")
        if m["T"] * m["N"] == 1:
            assert np.isnan(advn).all()
        else:
            np.testing.assert_allclose(advn, ref, rtol=1e-5, atol=1e-5, err_msg=name)


@pytest.mark.parametrize("T,N,p", [(24, 65536, 0.02), (24, 4096, 0.02), (1, 1000, 0.5), (40, 3001, 0.1),
                                   (33, 257, 0.05), (16, 512, 0.0), (8, 100003, 1.0), (32, 70000, 0.3)])
def test_random_vs_oracle(T, N, p, cuda_device):
    rng = np.random.default_rng(T * 1000 + N)
    values = rng.standard_normal((T, N), dtype=np.float32)
    rewards = rng.standard_normal((T, N), dtype=np.float32)
    dones = (rng.random((T, N)) < p).astype(np.uint8)
    last = rng.standard_normal(N, dtype=np.float32)
    ret, adv = _run(values, rewards, dones, last, 0.99, 0.95, False, cuda_device)
    oret, oadv = O.gae(values, rewards, dones, last, 0.99, 0.95)
    assert np.array_equal(ret, oret)
    assert np.array_equal(adv, oadv)
    _, advn = _run(values, rewards, dones, last, 0.99, 0.95, True, cuda_device)
    np.testing.assert_allclose(advn, O.adv_normalize(oadv), rtol=1e-5, atol=1e-5)


def test_full_size_properties(cuda_device):
    """C3 size (T=24, N=65536): normalised advantages have mean ~0 / std ~1, and the scan is
    idempotent and deterministic run to run (fixed reduction order)."""
    T, N = 24, 65536
    g = torch.Generator(device=cuda_device).manual_seed(5)
    v = torch.randn(T, N, 1, generator=g, device=cuda_device)
    r = torch.randn(T, N, 1, generator=g, device=cuda_device)
    d = (torch.rand(T, N, 1, generator=g, device=cuda_device) < 0.02).to(torch.uint8)
    lv = torch.randn(N, 1, generator=g, device=cuda_device)
    outs = []
    for _ in range(2):
        ret = torch.empty_like(v)
        adv = torch.empty_like(v)
        kernels.compute_returns(v, r, d, lv, 0.99, 0.95, True, ret, adv)
        outs.append((ret, adv))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    a = outs[0][1].double()
    assert abs(a.mean().item()) < 1e-6
    assert abs(a.std().item() - 1.0) < 1e-5
    # returns - values is the raw advantage: re-normalising it reproduces the normalised advantages
    raw = outs[0][0] - v
    ref = (raw - raw.double().mean().float()) / (raw.double().std().float() + 1e-8)
    assert torch.allclose(outs[0][1], ref, atol=1e-5)


# ---------------------------------------------------------------------------------------------------------------------
# rslrl_compute_returns_slots: its three forms (ABI 18) -- 0 scan + normaliser, 1 one launch with one env per lane,
# 2 one launch over LDS-staged tiles of 64 envs -- and the grid barrier's safety net
# ---------------------------------------------------------------------------------------------------------------------
def _slots_inputs(T, N, p, dev, seed):
    rng = np.random.default_rng(seed)
    f = lambda *s: torch.from_numpy(rng.standard_normal(s, dtype=np.float32)).to(dev)  # noqa: E731
    values, rewards, logp, last = f(T, N, 1), f(T, N, 1), f(T, N, 1), f(N, 1)
    dones = torch.from_numpy((rng.random((T, N, 1)) < p).astype(np.uint8)).to(dev)
    return values, rewards, dones, last, logp


def _slots_run(inp, form_cap=None, coop=None):
    values, rewards, dones, last, logp = inp
    T, N = values.shape[:2]
    old = {}
    try:
        if form_cap is not None:
            old["gae_form"] = kernels.debug_knob("gae_form", form_cap)
        if coop is not None:
            old["gae_coop"] = kernels.debug_knob("gae_coop", coop)
        L = kernels._lib.lib()
        ret, adv = torch.empty_like(values), torch.empty_like(values)
        slots = torch.full((T, N, 4), float("nan"), device=values.device)
        form = L.rslrl_compute_returns_slots_form(T, N, values.data_ptr(), rewards.data_ptr(), dones.data_ptr(),
                                                  logp.data_ptr(), ret.data_ptr(), adv.data_ptr())
        status = kernels.compute_returns_slots(values, rewards, dones, last, 0.99, 0.95, ret, adv, logp, slots)
        torch.cuda.synchronize()
        return form, ret, adv, slots, int(status.item())
    finally:
        for k, v in old.items():
            kernels.debug_knob(k, v)


@pytest.mark.parametrize("T,N,p", [(24, 65536, 0.02), (24, 16384, 0.02), (24, 4096, 0.02), (8, 64, 0.5),
                                   (16, 320, 0.1), (32, 131072, 0.3), (24, 131072, 0.02), (24, 1000, 0.02),
                                   (32, 8256, 1.0)])
def test_slots_forms_bit_identical(T, N, p, cuda_device):
    """Every form of compute_returns_slots gives the same bits as the two-launch form (returns, normalised advantages,
    the whole slot array); returns and raw advantages equal the oracle's.  Forms: 1 one env per lane in 256-thread
    blocks, 2 LDS-staged 64-env tiles (N % 64 == 0), 3 one env per lane in 64-thread blocks (N <= 65536), each forced
    through the knob (a form that does not apply runs the two-launch form)."""
    inp = _slots_inputs(T, N, p, cuda_device, T * N + 3)
    base = _slots_run(inp, form_cap=0)
    assert base[0] == 0 and base[4] == 0
    forms = {0}
    for cap in (1, 2, 3):
        for coop in (0, 1):
            form, ret, adv, slots, status = _slots_run(inp, form_cap=cap, coop=coop)
            assert form in (cap, 0) and status == 0
            forms.add(form)
            assert torch.equal(ret, base[1]) and torch.equal(adv, base[2]), (cap, coop, form)
            assert torch.equal(slots, base[3]), (cap, coop, form)
    auto = _slots_run(inp)
    assert torch.equal(auto[3], base[3])
    assert auto[0] != 0, "every shape here fits a one-launch form"
    if N % 64 == 0 and N <= 65536:
        assert 2 in forms and 3 in forms
    if N <= 65536:
        assert 3 in forms
    values, rewards, dones = (t.cpu().numpy().reshape(T, N) for t in inp[:3])
    oret, oadv = O.gae(values, rewards, dones, inp[3].cpu().numpy().reshape(N), 0.99, 0.95)
    assert np.array_equal(base[1].cpu().numpy().reshape(T, N), oret)
    np.testing.assert_allclose(base[2].cpu().numpy().reshape(T, N), O.adv_normalize(oadv), rtol=1e-5, atol=1e-5)
    assert len(forms) >= 2


def test_slots_golden_all_forms(golden_meta, cuda_device):
    """The reference's own GAE vectors through every form of compute_returns_slots: returns bit-exact, normalised
    advantages within 1e-5 of the reference's (its fp32 mean / std), slots = {value, log-prob, return, advantage}."""
    z = np.load(golden_path("gae.npz"))
    for name, m in sorted(golden_meta["gae"].items()):
        if m["T"] * m["N"] == 1:
            continue
        g = lambda k: z[f"{name}/{k}"]  # noqa: E731
        T, N = m["T"], m["N"]
        t = lambda a, *s: torch.from_numpy(np.ascontiguousarray(a)).reshape(*s).to(cuda_device)  # noqa: E731
        logp = torch.randn(T, N, 1, device=cuda_device)
        inp = (t(g("values"), T, N, 1), t(g("rewards"), T, N, 1), t(g("dones"), T, N, 1),
               t(g("last_values"), N, 1), logp)
        values, rewards, dones, last, _ = inp
        for cap in (0, 1, 2, 3):
            old = kernels.debug_knob("gae_form", cap)
            try:
                ret, adv = torch.empty_like(values), torch.empty_like(values)
                slots = torch.empty(T, N, 4, device=cuda_device)
                kernels.compute_returns_slots(values, rewards, dones, last, m["gamma"], m["lam"], ret, adv, logp, slots)
            finally:
                kernels.debug_knob("gae_form", old)
            assert np.array_equal(ret.cpu().numpy().reshape(T, N), g("returns")), (name, cap)
            np.testing.assert_allclose(adv.cpu().numpy().reshape(T, N), g("advantages_norm"), rtol=1e-5, atol=1e-5,
                                       err_msg=f"{name} form cap {cap}")
            assert torch.equal(slots, torch.cat([values, logp, ret, adv], dim=-1))


def test_slots_barrier_timeout_is_loud_and_recovers(cuda_device):
    """A grid-barrier wait that gives up (forced: spin limit 0, so every block that is not the last to arrive stops
    waiting at once) raises the workspace's status word and writes NaN advantages instead of normalising with partial
    statistics; raise_on_gae_status raises and clears the word, and the next call (normal limit) is bit-exact again --
    the late blocks re-armed the ticket.  Both one-launch forms, plain and cooperative launches."""
    for N, fm in ((65536, 2), (65536 + 100, 1), (16384, 3)):  # each one-launch form
        inp = _slots_inputs(24, N, 0.02, cuda_device, 11)
        base = _slots_run(inp, form_cap=0)
        for coop in (0, 1):
            old = kernels.debug_knob("gae_spin_limit", 0)
            try:
                form, ret, adv, slots, status = _slots_run(inp, form_cap=fm, coop=coop)
            finally:
                kernels.debug_knob("gae_spin_limit", old)
            assert form == fm
            assert status != 0, "no block timed out with a zero spin limit"
            assert torch.isnan(adv).any() and torch.equal(ret, base[1])
            values, rewards, dones, last, logp = inp
            ws = kernels._gae_workspace(values.device, 24, N)
            word = kernels.gae_status_word(ws)
            with pytest.raises(kernels.GAEBarrierTimeout):
                kernels.raise_on_gae_status(word)
            assert int(word.item()) == 0
            form, ret, adv, slots, status = _slots_run(inp, form_cap=fm, coop=coop)
            assert status == 0 and torch.equal(adv, base[2]) and torch.equal(slots, base[3])
            bar = ws[kernels._lib.lib().rslrl_compute_returns_status_offset() - 8:].view(torch.int32)[:2].tolist()
            assert bar[0] == 0, bar  # ticket re-armed


def test_update_raises_on_gae_barrier_timeout(cuda_device):
    """PPO.update reads compute_returns' status word with its loss statistics and raises GAEBarrierTimeout when the
    grid barrier gave up (forced through the spin-limit knob), instead of returning losses of NaN advantages; the
    storage is cleared and the word reset, so the runner object stays usable (its parameters are NaN by then)."""
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.runners import OnPolicyRunner

    torch.manual_seed(0)
    env = SyntheticVecEnv(4096, 16, 4, device=cuda_device, seed=0)
    cfg = {
        "num_steps_per_env": 24, "save_interval": 50, "obs_groups": {"policy": ["policy"]},
        "policy": {"class_name": "ActorCritic", "actor_hidden_dims": [64, 64], "critic_hidden_dims": [64, 64],
                   "activation": "elu", "init_noise_std": 1.0},
        "algorithm": {"class_name": "PPO", "num_learning_epochs": 1, "num_mini_batches": 2},
    }
    runner = OnPolicyRunner(env, cfg, log_dir=None, device=str(cuda_device))
    runner.learn(1)  # normal
    old = kernels.debug_knob("gae_spin_limit", 0)
    try:
        with pytest.raises(kernels.GAEBarrierTimeout):
            runner.learn(1)
    finally:
        kernels.debug_knob("gae_spin_limit", old)
    assert runner.alg.storage.step == 0 and runner.alg.storage.gae_status is None


def test_slots_mixed_grid_sizes_share_a_workspace(cuda_device):
    """Calls of different grid sizes (and forms) on one stream share the workspace's barrier words: each call moves
    every group's generation word, so a call after a smaller grid still completes its barrier (no time-out, no NaN) and
    matches the two-launch form bit for bit."""
    cases = [(24, 65636), (24, 65536), (24, 4096), (24, 65636), (24, 131072), (8, 1000), (24, 65536), (32, 16384)]
    inputs = {c: _slots_inputs(c[0], c[1], 0.02, cuda_device, c[1] + c[0]) for c in set(cases)}
    base = {c: _slots_run(inputs[c], form_cap=0) for c in set(cases)}
    for c in cases + cases[::-1]:
        for fm in (None, 1, 2, 3):
            form, ret, adv, slots, status = _slots_run(inputs[c], form_cap=fm)
            assert status == 0, (c, form)
            assert torch.equal(adv, base[c][2]) and torch.equal(slots, base[c][3]), (c, form)
