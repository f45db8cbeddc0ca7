"""Fused HIP PPO loss (rslrl_ppo_loss_fwd_bwd) vs the reference's captured loss/KL/gradients and vs the
oracle on random inputs.  Tolerance: rtol 1e-5 (relative to the tensor's max magnitude for gradients),
as north_star states for floating point."""

import numpy as np
import pytest
import torch

from conftest import golden_path
from oracle import ppo_oracle as O
from rsl_rl_amd import kernels

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _rel_err(a, ref):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(a - ref)) / (np.max(np.abs(ref)) + 1e-30))


def _close_but_rare_flips(a, ref, B, rtol=RTOL):
    a = np.asarray(a, np.float64).reshape(B, -1)
    ref = np.asarray(ref, np.float64).reshape(B, -1)
    bad_rows = (np.abs(a - ref) > rtol * (np.max(np.abs(ref)) + 1e-30)).any(axis=1)
    assert bad_rows.sum() <= max(1, int(1e-5 * B)), int(bad_rows.sum())


def _kw(m):
    kw = m["ppo_kw"]
    return dict(clip_param=kw.get("clip_param", 0.2), value_loss_coef=kw.get("value_loss_coef", 1.0),
                entropy_coef=kw.get("entropy_coef", 0.01), use_clipped_value_loss=kw.get("use_clipped_value_loss", True),
                compute_kl=m["adaptive"], normalize_advantage=kw.get("normalize_advantage_per_mini_batch", False))


def test_golden_cases(golden_meta, cuda_device):
    for name, m in sorted(golden_meta["loss"].items()):
        z = np.load(golden_path(f"loss_{name}.npz"))
        state_dep = m["policy_kw"].get("state_dependent_std", False)
        for j in range(m["num_batches"]):
            g = lambda k: torch.from_numpy(z[f"mb{j}/{k}"]).to(cuda_device)  # noqa: E731
            sigma_rows = g("sigma")
            # shared sigma: the policy's [A] std (every row of the expanded sigma is identical)
            sigma = sigma_rows if state_dep else sigma_rows[0].contiguous()
            stats, gmu, gsig, gv = kernels.ppo_loss_fwd_bwd(
                g("mu"), sigma, g("V"), g("actions"), g("old_logp"), g("advantages"), g("target_values"),
                g("returns"), g("old_mu"), g("old_sigma"), **_kw(m))
            torch.cuda.synchronize()
            assert _rel_err(gmu.cpu(), z[f"mb{j}/dmu"]) < RTOL, (name, j)
            assert _rel_err(gv.cpu().reshape(-1), z[f"mb{j}/dV"].reshape(-1)) < RTOL, (name, j)
            dsig_ref = z[f"mb{j}/dsigma"]
            if state_dep:
                assert _rel_err(gsig.cpu(), dsig_ref) < RTOL, (name, j)
            else:
                assert _rel_err(gsig.cpu(), dsig_ref.astype(np.float64).sum(0)) < RTOL, (name, j)
            s = stats.cpu().numpy()
            if m["adaptive"]:
                kl = float(z[f"mb{j}/kl_mean"])
                assert abs(s[kernels.STATS_KL] - kl) <= RTOL * abs(kl) + 1e-9, (name, j)
            if m["num_batches"] == 1:
                ld = m["loss_dict"]
                assert abs(s[kernels.STATS_SURROGATE] - ld["surrogate"]) <= RTOL * abs(ld["surrogate"]) + 1e-7
                assert abs(s[kernels.STATS_VALUE] - ld["value_function"]) <= RTOL * abs(ld["value_function"]) + 1e-7
                assert abs(s[kernels.STATS_ENTROPY] - ld["entropy"]) <= RTOL * abs(ld["entropy"]) + 1e-7


@pytest.mark.parametrize("B,A,shared,kw", [
    (393216, 12, True, {}),
    (98304, 12, False, {}),
    (1001, 3, True, {"use_clipped_value_loss": False}),
    (5000, 7, False, {"normalize_advantage": True}),
    (4099, 16, True, {"compute_kl": False, "clip_param": 0.1}),
    (777, 33, True, {}),
    (300, 64, False, {"entropy_coef": 0.0}),
    (1, 4, True, {}),
    (4097, 8, False, {}),
    (70000, 4, True, {"compute_kl": False}),
])
@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_random_vs_oracle(B, A, shared, kw, kernel, cuda_device, monkeypatch):
    # RSLRL_LOSS_KERNEL is read per call by the library (quad layout: A % 4 == 0 and A <= 16)
    monkeypatch.setenv("RSLRL_LOSS_KERNEL", kernel)
    rng = np.random.default_rng(B + A)
    mu = rng.standard_normal((B, A), dtype=np.float32)
    sig_vec = rng.uniform(0.5, 1.5, A).astype(np.float32)
    sig = np.broadcast_to(sig_vec, (B, A)).copy() if shared else rng.uniform(0.5, 1.5, (B, A)).astype(np.float32)
    x = rng.standard_normal((B, A), dtype=np.float32)
    omu = rng.standard_normal((B, A), dtype=np.float32)
    osig = rng.uniform(0.5, 1.5, (B, A)).astype(np.float32)
    # logp of the actions under (mu, sig) + N(0, 0.3^2), as in SURVEY.md §8d
    logp = (-(x - mu) ** 2 / (2 * sig ** 2) - np.log(sig) - 0.9189385).sum(-1)
    old_logp = (logp + 0.3 * rng.standard_normal(B)).astype(np.float32)
    adv = rng.standard_normal(B, dtype=np.float32)
    tv = rng.standard_normal(B, dtype=np.float32)
    V = (tv + 0.3 * rng.standard_normal(B)).astype(np.float32)
    R = rng.standard_normal(B, dtype=np.float32)
    okw = dict(kw)
    if "normalize_advantage" in okw:
        okw["normalize_advantage_per_mini_batch"] = okw.pop("normalize_advantage")
    ref = O.ppo_loss(mu, sig, V, x, old_logp, adv, tv, R, omu, osig, **okw)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda_device)  # noqa: E731
    sigma = t(sig_vec) if shared else t(sig)
    stats, gmu, gsig, gv = kernels.ppo_loss_fwd_bwd(t(mu), sigma, t(V), t(x), t(old_logp), t(adv), t(tv), t(R),
                                                    t(omu), t(osig), **kw)
    torch.cuda.synchronize()
    # the oracle's numpy exp/log and the device's differ by <= 1 ulp, which can move a sample whose ratio
    # sits exactly on a clip bound to the other branch; allow that for <= 1e-5 of the samples.  The
    # A-term fp32 log-prob sum is rounded in a different order by numpy (pairwise) and the kernel
    # (sequential): its error grows ~sqrt(A) ulp(|logp|), so for A > 16 the bound is 5e-5.
    rtol = RTOL if A <= 16 else 5e-5
    _close_but_rare_flips(gmu.cpu().numpy(), ref["dmu"], B, rtol)
    _close_but_rare_flips(gv.cpu().numpy(), ref["dV"], B, rtol)
    if shared:
        dsig_ref = ref["dsigma"].astype(np.float64).sum(0)
        assert _rel_err(gsig.cpu(), dsig_ref) < (1e-4 if B > 100000 else rtol)
    else:
        _close_but_rare_flips(gsig.cpu().numpy(), ref["dsigma"], B, rtol)
    s = stats.cpu().numpy().astype(np.float64)
    for k, col in (("surrogate", kernels.STATS_SURROGATE), ("value_function", kernels.STATS_VALUE),
                   ("entropy", kernels.STATS_ENTROPY), ("loss", kernels.STATS_LOSS)):
        assert abs(s[col] - ref[k]) <= rtol * abs(ref[k]) + 1e-6, k
    if kw.get("compute_kl", True):
        assert abs(s[kernels.STATS_KL] - ref["kl_mean"]) <= rtol * abs(ref["kl_mean"]) + 1e-7


def test_autograd_function_matches_torch(cuda_device):
    """PPOLossFunction through autograd == the reference expressions evaluated by torch autograd."""
    torch.manual_seed(0)
    B, A = 2048, 6
    dev = cuda_device
    mu = torch.randn(B, A, device=dev, requires_grad=True)
    std = (0.5 + torch.rand(A, device=dev)).requires_grad_()
    V = torch.randn(B, 1, device=dev, requires_grad=True)
    x, omu = torch.randn(B, A, device=dev), torch.randn(B, A, device=dev)
    osig = 0.5 + torch.rand(B, A, device=dev)
    old_logp, adv, tv, R = (torch.randn(B, 1, device=dev) for _ in range(4))
    loss, _ = kernels.PPOLossFunction.apply(mu, std, V, x, old_logp, adv, tv, R, omu, osig, 0.2, 1.0, 0.01,
                                            True, True, False)
    loss.backward()
    g_ours = [mu.grad.clone(), std.grad.clone(), V.grad.clone()]
    for p in (mu, std, V):
        p.grad = None
    d = torch.distributions.Normal(mu, std.expand_as(mu))
    logp = d.log_prob(x).sum(-1)
    ratio = torch.exp(logp - old_logp.squeeze())
    s1 = -adv.squeeze() * ratio
    s2 = -adv.squeeze() * torch.clamp(ratio, 0.8, 1.2)
    vc = tv + (V - tv).clamp(-0.2, 0.2)
    ref = (torch.max(s1, s2).mean() + torch.max((V - R).pow(2), (vc - R).pow(2)).mean()
           - 0.01 * d.entropy().sum(-1).mean())
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    for a, b in zip(g_ours, [mu.grad, std.grad, V.grad]):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item() + 1e-9


@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_value_gradient_into_padded_column(kernel, cuda_device, monkeypatch):
    """grad_values as column 0 of a [B, 4] buffer (row stride 4, the value head's padded operand): the same bits
    as the contiguous [B] output; the other columns are left as they were."""
    monkeypatch.setenv("RSLRL_LOSS_KERNEL", kernel)
    torch.manual_seed(3)
    B, A = 5000, 12
    d = cuda_device
    mu, x, omu = (torch.randn(B, A, device=d) for _ in range(3))
    osig = 0.5 + torch.rand(B, A, device=d)
    sigma = 0.5 + torch.rand(A, device=d)
    V, old_logp, adv, tv, R = (torch.randn(B, 1, device=d) for _ in range(5))
    args = (mu, sigma, V, x, old_logp, adv, tv, R, omu, osig)
    _, _, _, gv = kernels.ppo_loss_fwd_bwd(*args)
    pad = torch.full((B, 4), 7.0, device=d)
    _, _, _, gv2 = kernels.ppo_loss_fwd_bwd(*args, grad_values=pad[:, :1])
    torch.cuda.synchronize()
    assert gv2.data_ptr() == pad.data_ptr()
    assert torch.equal(pad[:, 0], gv.reshape(-1)) and (pad[:, 1:] == 7.0).all()


@pytest.mark.parametrize("B,perturb", [(393216, 0), (393216, 37), (4099, 5), (64, 64)])
def test_shared_sigma_kl_fast_path_bit_exact(B, perturb, cuda_device, monkeypatch):
    """The quad kernel's shared-sigma KL (per-action log term, division by the constant 2 sigma^2 through the
    correctly rounded reciprocal + fma correction) gives the same bits as the reference's full expression
    (RSLRL_KL_FAST=0), with old sigmas as a rollout stores them (one value per action) plus `perturb` rows whose
    old sigma or mean differs (those elements take the full expression in the fast kernel too); and the KL
    matches the oracle."""
    monkeypatch.setenv("RSLRL_LOSS_KERNEL", "quad")
    A = 12
    rng = np.random.default_rng(B + perturb)
    mu = rng.standard_normal((B, A), dtype=np.float32)
    sig_vec = rng.uniform(0.3, 1.5, A).astype(np.float32)
    old_vec = (sig_vec * rng.uniform(0.9, 1.1, A)).astype(np.float32)
    osig = np.broadcast_to(old_vec, (B, A)).copy()
    omu = (mu + 0.05 * rng.standard_normal((B, A))).astype(np.float32)
    rows = rng.choice(B, size=perturb, replace=False) if perturb else np.zeros(0, np.int64)
    osig[rows[: perturb // 2]] *= np.float32(1.25)
    omu[rows[perturb // 2:]] = np.float32(3e19)  # (old mu - mu)^2 beyond the fast path's range
    x = rng.standard_normal((B, A), dtype=np.float32)
    old_logp = rng.standard_normal(B).astype(np.float32) - 10.0
    adv, tv, V, R = (rng.standard_normal(B, dtype=np.float32) for _ in range(4))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda_device)  # noqa: E731
    args = (t(mu), t(sig_vec), t(V), t(x), t(old_logp), t(adv), t(tv), t(R), t(omu), t(osig))
    out = {}
    for fast in ("1", "0"):
        monkeypatch.setenv("RSLRL_KL_FAST", fast)
        stats, gmu, gsig, gv = kernels.ppo_loss_fwd_bwd(*args)
        torch.cuda.synchronize()
        out[fast] = (stats.cpu().clone(), gmu.cpu().clone(), gsig.cpu().clone(), gv.cpu().clone())
    for a, b in zip(out["1"], out["0"]):
        assert torch.equal(a, b)
    if perturb == 0:
        ref = O.ppo_loss(mu, np.broadcast_to(sig_vec, (B, A)), V, x, old_logp, adv, tv, R, omu, osig)
        kl = float(out["1"][0][kernels.STATS_KL])
        assert abs(kl - ref["kl_mean"]) <= RTOL * abs(ref["kl_mean"]) + 1e-7


def test_quad_kernel_pipeline_depth_bit_identical(cuda_device, monkeypatch):
    """RSLRL_LOSS_DEPTH 2 (two tiles in flight per wave) computes every tile the same way: identical bits."""
    monkeypatch.setenv("RSLRL_LOSS_KERNEL", "quad")
    torch.manual_seed(5)
    B, A, d = 100003, 12, cuda_device
    mu, x, omu = (torch.randn(B, A, device=d) for _ in range(3))
    osig = (0.5 + torch.rand(A, device=d)).expand(B, A).contiguous()
    sigma = 0.5 + torch.rand(A, device=d)
    V, old_logp, adv, tv, R = (torch.randn(B, 1, device=d) for _ in range(5))
    out = []
    for depth in ("1", "2"):
        monkeypatch.setenv("RSLRL_LOSS_DEPTH", depth)
        res = kernels.ppo_loss_fwd_bwd(mu, sigma, V, x, old_logp, adv, tv, R, omu, osig)
        torch.cuda.synchronize()
        out.append([t.clone() for t in res])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_launch_bound_event_timing(cuda_device, monkeypatch):
    """rslrl_launch_timing_*: while armed, each quad-kernel launch carries its own event pair (one record per
    launch, up to the capacity); the results are the same bits as an unarmed launch; each bound duration is positive
    and no longer than the marker span around the C-ABI call; disarming keeps the records readable."""
    monkeypatch.setenv("RSLRL_LOSS_KERNEL", "quad")
    torch.manual_seed(9)
    B, A, d = 393216, 12, cuda_device
    mu, x, omu = (torch.randn(B, A, device=d) for _ in range(3))
    osig = (0.5 + torch.rand(A, device=d)).expand(B, A).contiguous()
    sigma = 0.5 + torch.rand(A, device=d)
    V, old_logp, adv, tv, R = (torch.randn(B, 1, device=d) for _ in range(5))
    args = (mu, sigma, V, x, old_logp, adv, tv, R, omu, osig)
    plain = [t.clone() for t in kernels.ppo_loss_fwd_bwd(*args)]
    kernels.timer.arm_launch_events(3)
    try:
        spans = []
        for _ in range(4):  # the 4th launch is past the capacity: unbound
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = kernels.ppo_loss_fwd_bwd(*args)
            e.record()
            spans.append((s, e))
        torch.cuda.synchronize()
    finally:
        kernels.timer.disarm_launch_events()
    for a, b in zip(plain, out):
        assert torch.equal(a, b)
    total_ms, n = kernels.timer.launch_events()
    assert n == 3
    span_ms = sum(s.elapsed_time(e) for s, e in spans[:3])
    assert 0.0 < total_ms <= span_ms * 1.001
