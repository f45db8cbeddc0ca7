"""The actor's fused head (rslrl_actor_head_fwd_bwd: last hidden layer + the 12-wide output layer + the whole PPO loss +
the output layer's backward in one launch) against the separate launches it replaces: the fused output-layer forward
(linear_fwd_out_ex), the PPO loss kernel (ppo_loss_fwd_bwd) and the output-layer backward (linear_dgrad_elu_wgrad).
mu and d loss / d mu are bit-identical; the loss statistics and d sigma fold per 128-row tile (fp64, another
partition: fp32-close); dz comes from x6 products of d mu and W_out where the separate backward runs an fp32 FMA chain
(fp32-close); the output layer's weight and bias gradients sum the rows in another order (fp32-close).  Then a whole
PPO.update() with and without it."""

import numpy as np
import pytest
import torch

from rsl_rl_amd import _lib, kernels
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu

A = 12


def _problem(M, dev, seed, old_sigma_per_row=False):
    g = torch.Generator(device=dev).manual_seed(seed)
    K = N = 256
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x = torch.nn.functional.elu(r(M, K))
    w, b = r(N, K) / 16, r(N) * 0.1
    wo, bo = r(A, N) / 16, r(A) * 0.1
    sigma = torch.rand(A, device=dev, generator=g) * 0.5 + 0.5
    old_sigma = (sigma * (1.0 + 0.1 * torch.rand(A, device=dev, generator=g))).expand(M, A).contiguous()
    if old_sigma_per_row:  # every third row's sigma_old differs from row 0's bits: the per-element KL expression
        old_sigma[1::3] *= 1.0 + 0.05 * torch.rand(old_sigma[1::3].shape, device=dev, generator=g)
    batch = dict(actions=r(M, A), old_log_prob=r(M, 1) - 8.0, advantages=r(M, 1), target_values=r(M, 1) * 0.3,
                 returns=r(M, 1), old_mu=r(M, A) * 0.1, old_sigma=old_sigma)
    values = r(M, 1) * 0.3
    return x, w, b, wo, bo, sigma, values, batch


def _separate(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, clipped, kl):
    N = w.shape[0]
    h, mu = fused_mlp.linear_fwd_out_ex(x, b, N, img, _lib.ARITH_X6, None, bo, out_img, store_h=True)
    stats, gmu, gsig, _ = kernels.ppo_loss_fwd_bwd(
        mu, sigma, values, batch["actions"], batch["old_log_prob"], batch["advantages"], batch["target_values"],
        batch["returns"], batch["old_mu"], batch["old_sigma"], clip_param=0.2, value_loss_coef=1.0,
        entropy_coef=0.01, use_clipped_value_loss=clipped, compute_kl=kl)
    dz, _, dw, db = fused_mlp.linear_dgrad_elu_wgrad(gmu, wo, h, img_t)
    return mu, stats.clone(), gmu, gsig.clone(), dz, dw, db


def _fused(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, clipped, kl):
    M, N = x.shape[0], w.shape[0]
    dev = x.device
    head = fused_mlp.ActorHead(batch["actions"], batch["old_log_prob"], batch["advantages"], batch["target_values"],
                               batch["returns"], batch["old_mu"], batch["old_sigma"], sigma, clip_param=0.2,
                               value_loss_coef=1.0, entropy_coef=0.01, use_clipped=clipped, compute_kl=kl,
                               grad_sigma=torch.empty(A, device=dev), stats=torch.empty(8, device=dev),
                               grad_mu=torch.empty(M, A, device=dev))
    head.values = values
    res = fused_mlp.actor_head_fwd_bwd(x, b, N, img, bo, out_img, img_t, head)
    assert res is not None and head.done
    dz, mu, wpart = res
    folds = fused_mlp._FoldBatch()
    dwb = torch.empty(A * N + A, device=dev)
    folds.add(wpart, wpart.shape[0], wpart.shape[1], dwb, A * N + A)
    folds.run(dev)
    return mu, head.stats, head.grad_mu, head.grad_sigma, dz, dwb[:A * N].view(A, N), dwb[A * N:]


def _close(a, b, rtol):
    scale = float(b.abs().max()) + 1e-30
    return torch.allclose(a, b, rtol=rtol, atol=rtol * 0.1 * scale)


@pytest.mark.parametrize("M,clipped,kl", [(4096, True, True), (4096, False, False), (98304, True, True),
                                          (393216, True, True), (786432, True, True)])
def test_actor_head_matches_separate_launches(M, clipped, kl, cuda_device):
    """786,432 rows (C4's 131,072 envs on one GPU: 6,144 tiles) fold the loss partials in groups of 128 tiles."""
    dev = cuda_device
    x, w, b, wo, bo, sigma, values, batch = _problem(M, dev, 21 + M)
    img, out_img, img_t = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT), (wo, True)])
    ref = _separate(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, clipped, kl)
    got = _fused(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, clipped, kl)
    torch.cuda.synchronize()
    mu_r, st_r, gmu_r, gs_r, dz_r, dw_r, db_r = ref
    mu, st, gmu, gs, dz, dw, db = got
    assert torch.equal(mu, mu_r)
    assert torch.equal(gmu, gmu_r)
    assert torch.allclose(st[:5], st_r[:5], rtol=2e-6, atol=1e-9), (st, st_r)
    assert torch.equal(st[5:], st_r[5:])
    assert torch.allclose(gs, gs_r, rtol=1e-5, atol=1e-9)
    assert _close(dz, dz_r, 1e-5)
    assert _close(dw, dw_r, 1e-5)
    assert _close(db, db_r, 1e-5)
    # the launch re-arms its fold tickets: a second run gives the same bits
    again = _fused(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, clipped, kl)
    torch.cuda.synchronize()
    for u, v in zip(got, again):
        assert torch.equal(u, v)


@pytest.mark.parametrize("case", ["old_sigma_per_row", "kl_fast_off"])
def test_actor_head_kl_fallbacks_match_loss_kernel(case, cuda_device, monkeypatch):
    """The fused head's KL on rows whose sigma_old is not sample 0's (the per-element fallback of the per-action-constant
    fast path) and with the fast path switched off (RSLRL_KL_FAST=0, read per launch by both kernels): the KL
    (stats[4]) and every other loss output as ppo_loss_fwd_bwd's on the same inputs."""
    dev, M = cuda_device, 16384
    if case == "kl_fast_off":
        monkeypatch.setenv("RSLRL_KL_FAST", "0")
    x, w, b, wo, bo, sigma, values, batch = _problem(M, dev, 77, old_sigma_per_row=case == "old_sigma_per_row")
    img, out_img, img_t = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT), (wo, True)])
    mu_r, st_r, gmu_r, gs_r, dz_r, dw_r, db_r = _separate(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t,
                                                          True, True)
    mu, st, gmu, gs, dz, dw, db = _fused(x, w, b, wo, bo, sigma, values, batch, img, out_img, img_t, True, True)
    torch.cuda.synchronize()
    assert torch.equal(mu, mu_r) and torch.equal(gmu, gmu_r)
    assert torch.allclose(st[:5], st_r[:5], rtol=2e-6, atol=1e-9), (st, st_r)
    assert float(st[4]) > 0.0  # the KL of these inputs is not the rollout-consistent ~0
    assert torch.allclose(gs, gs_r, rtol=1e-5, atol=1e-9)
    assert _close(dz, dz_r, 1e-5) and _close(dw, dw_r, 1e-5) and _close(db, db_r, 1e-5)


def test_actor_head_declines_unsupported(cuda_device):
    """Partial tiles or another action count: nothing launched, the caller keeps the separate launches."""
    dev = cuda_device
    x, w, b, wo, bo, sigma, values, batch = _problem(1000, dev, 5)
    img, out_img, img_t = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT), (wo, True)])
    head = fused_mlp.ActorHead(batch["actions"], batch["old_log_prob"], batch["advantages"], batch["target_values"],
                               batch["returns"], batch["old_mu"], batch["old_sigma"], sigma, clip_param=0.2,
                               value_loss_coef=1.0, entropy_coef=0.01, use_clipped=True, compute_kl=True,
                               grad_sigma=torch.empty(A, device=dev), stats=torch.empty(8, device=dev))
    head.values = values
    assert fused_mlp.actor_head_fwd_bwd(x, b, 256, img, bo, out_img, img_t, head) is None
    assert not head.done


@pytest.mark.parametrize("noise_std_type", ["scalar", "log"])
def test_update_with_actor_head_matches_separate_launches(noise_std_type, cuda_device, monkeypatch):
    """PPO.update() on one storage with the fused actor head and with the separate launches (RSLRL_ACTOR_HEAD off; the
    critic's fused head on in both): the same learning-rate trace and loss statistics, and parameters within fp32
    accumulation-order noise."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    dev = cuda_device
    T, N, O = 8, 2048, 48  # 16384 rows: 4 mini-batches of 4096 (32 tiles each)
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    rng = np.random.default_rng(4)
    data = {k: rng.standard_normal(s).astype(np.float32) for k, s in
            (("obs", (T, N, O)), ("rewards", (T, N, 1)), ("values", (T, N, 1)), ("logp", (T, N, 1)),
             ("mu", (T, N, A)), ("actions", (T, N, A)), ("last", (N, O)))}
    results = []
    for fused in (True, False):
        monkeypatch.setattr(fused_mlp, "_ACTOR_HEAD", fused)
        calls = []
        real = fused_mlp.actor_head_fwd_bwd
        monkeypatch.setattr(fused_mlp, "actor_head_fwd_bwd", lambda *a, **k: calls.append(1) or real(*a, **k))
        torch.manual_seed(0)
        pol = ActorCritic(obs0, groups, A, actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256],
                          noise_std_type=noise_std_type)
        alg = PPO(pol, num_learning_epochs=2, num_mini_batches=4, device=dev, desired_kl=0.01)
        alg.init_storage("rl", N, T, obs0, [A])
        st = alg.storage
        st.observations["policy"].copy_(torch.from_numpy(data["obs"]))
        st.rewards.copy_(torch.from_numpy(data["rewards"]))
        st.values.copy_(torch.from_numpy(data["values"]))
        st.actions_log_prob.copy_(torch.from_numpy(data["logp"]) - 10.0)
        st.mu.copy_(torch.from_numpy(data["mu"]) * 0.1)
        st.sigma.copy_(torch.ones(T, N, A))
        st.actions.copy_(torch.from_numpy(data["actions"]))
        st.dones.zero_()
        st.step = T
        with torch.inference_mode():
            alg.compute_returns({"policy": torch.from_numpy(data["last"]).to(dev)})
        st.perm_generator = torch.Generator().manual_seed(1)
        loss = alg.update()
        assert len(calls) == (8 if fused else 0)
        results.append((loss, alg.learning_rate, {k: v.detach().clone() for k, v in pol.state_dict().items()}))
    (l1, lr1, p1), (l0, lr0, p0) = results
    assert lr1 == lr0
    for k in l0:
        assert np.isclose(l1[k], l0[k], rtol=1e-4, atol=1e-7), k
    for k in p0:
        assert torch.allclose(p1[k], p0[k], rtol=1e-4, atol=2e-6), k
