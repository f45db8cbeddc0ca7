"""The critic's fused head (rslrl_value_head_fwd_bwd: last hidden layer + value head + d(value loss)/dV + the value
head's backward in one launch) against the separate launches it replaces: the fused output-layer forward
(linear_fwd_out_ex), the PPO loss kernel's d/dV (ppo_loss_fwd_bwd) and the output-layer backward
(linear_dgrad_elu_wgrad).  Values and the last hidden layer's dz are bit-identical; the head's weight and bias
gradients are sums over the rows in another order (fp32-close).  Then a whole PPO.update() with and without it."""

import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from rsl_rl_amd import _lib, kernels
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu


def L_rows(M, with_colsum=False):
    return _lib.lib().rslrl_value_head_partial_rows(M, int(with_colsum))


def _stream_form():
    """True when this process runs the head's streaming form: one partial row per slice (256 at C3, not 3072)."""
    return L_rows(393216) < 393216 // 128


def _loss_dv(values, tv, ret, clipped, clip, coef, dev, g):
    """The loss kernel's d loss / dV for these values (random actor-side inputs: they do not enter d/dV)."""
    B, A = values.shape[0], 12
    mu = torch.randn(B, A, device=dev, generator=g)
    sigma = torch.rand(A, device=dev, generator=g) + 0.5
    z = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    _, _, _, g_value = kernels.ppo_loss_fwd_bwd(
        mu, sigma, values, z(B, A), z(B, 1), z(B, 1), tv, ret, z(B, A), sigma.expand(B, A).contiguous(),
        clip_param=clip, value_loss_coef=coef, use_clipped_value_loss=clipped)
    return g_value.reshape(B, 1).contiguous()


@pytest.mark.parametrize("M,clipped", [(4096, True), (4096, False), (98304, True), (393216, True)])
def test_value_head_matches_separate_launches(M, clipped, cuda_device):
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(11 + M)
    K = N = 256
    x = torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g))
    w = torch.randn(N, K, device=dev, generator=g) / 16
    b = torch.randn(N, device=dev, generator=g) * 0.1
    wo = torch.randn(1, N, device=dev, generator=g) / 16
    bo = torch.randn(1, device=dev, generator=g) * 0.1
    tv = torch.randn(M, 1, device=dev, generator=g) * 0.3
    ret = torch.randn(M, 1, device=dev, generator=g)
    clip, coef = 0.2, 1.0
    img, out_img, img_t = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT), (wo, True)])
    # separate launches: forward, the loss kernel's d/dV, the output-layer backward
    h, y_ref = fused_mlp.linear_fwd_out_ex(x, b, N, img, _lib.ARITH_X6, None, bo, out_img, store_h=True)
    dv = _loss_dv(y_ref, tv, ret, clipped, clip, coef, dev, g)
    dz_ref, _, dw_ref, db_ref = fused_mlp.linear_dgrad_elu_wgrad(dv, wo, h, img_t)
    # fused
    head = fused_mlp.ValueHead(tv, ret, clip, coef, clipped)
    res = fused_mlp.value_head_fwd_bwd(x, b, N, img, bo, out_img, wo, head)
    assert res is not None
    dz, y, wpart = res
    folds = fused_mlp._FoldBatch()
    dwb = torch.empty(N + 1, device=dev)
    folds.add(wpart, wpart.shape[0], wpart.shape[1], dwb, N + 1)
    folds.run(dev)
    torch.cuda.synchronize()
    if _stream_form():
        # the streaming form (one partial row per slice) sums V over 8 waves x 32 columns (fp32 reassociation): V, dV
        # and dz to rounding
        assert wpart.shape[0] == L_rows(M)
        assert torch.allclose(y, y_ref, rtol=1e-5, atol=1e-6 * float(y_ref.abs().max()))
        assert torch.allclose(dz, dz_ref, rtol=1e-4, atol=1e-5 * float(dz_ref.abs().max()))
    else:
        assert torch.equal(y, y_ref)
        assert torch.equal(dz, dz_ref)
    scale = float(dw_ref.abs().max()) + 1e-30
    assert torch.allclose(dwb[:N].view(1, N), dw_ref, rtol=1e-5, atol=1e-6 * scale)
    assert torch.allclose(dwb[N:], db_ref, rtol=1e-5, atol=1e-6 * float(db_ref.abs().max() + 1e-30))


def test_value_head_declines_partial_tiles(cuda_device):
    """A row count that is not a whole number of 128-row tiles: nothing launched, the caller keeps the separate
    launches."""
    dev = cuda_device
    M, K, N = 1000, 256, 256
    x = torch.randn(M, K, device=dev)
    w, b = torch.randn(N, K, device=dev) / 16, torch.zeros(N, device=dev)
    wo, bo = torch.randn(1, N, device=dev) / 16, torch.zeros(1, device=dev)
    img, out_img = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT)])
    head = fused_mlp.ValueHead(torch.zeros(M, 1, device=dev), torch.zeros(M, 1, device=dev), 0.2, 1.0, True)
    assert fused_mlp.value_head_fwd_bwd(x, b, N, img, bo, out_img, wo, head) is None


def test_update_with_value_head_matches_separate_launches(cuda_device, monkeypatch):
    """PPO.update() on one storage with the fused critic head and with the separate launches (RSLRL_VALUE_HEAD off):
    the same learning-rate trace and loss statistics, and parameters within fp32 accumulation-order noise."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    dev = cuda_device
    T, N, O, A = 8, 2048, 48, 12  # 16384 rows: 4 mini-batches of 4096 (32 tiles each)
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    rng = np.random.default_rng(3)
    data = {k: rng.standard_normal(s).astype(np.float32) for k, s in
            (("obs", (T, N, O)), ("rewards", (T, N, 1)), ("values", (T, N, 1)), ("logp", (T, N, 1)),
             ("mu", (T, N, A)), ("actions", (T, N, A)), ("last", (N, O)))}
    results = []
    for fused in (True, False):
        monkeypatch.setattr(fused_mlp, "_VALUE_HEAD", fused)
        torch.manual_seed(0)
        pol = ActorCritic(obs0, groups, A, actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256])
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
        results.append((loss, alg.learning_rate, {k: v.detach().clone() for k, v in pol.state_dict().items()}))
    (l1, lr1, p1), (l0, lr0, p0) = results
    assert lr1 == lr0
    for k in l0:
        assert np.isclose(l1[k], l0[k], rtol=1e-4, atol=1e-7), k
    for k in p0:
        assert torch.allclose(p1[k], p0[k], rtol=1e-4, atol=2e-6), k


def test_value_head_other_form_in_a_child(cuda_device):
    """The head's other form (RSLRL_VALUE_HEAD_STREAM, read once per process: the tiled kernel or the streaming main
    loop) against the same separate launches, in a child process: the tiled form bit-exact, the streaming form's V / dz
    to rounding and its per-slice partial rows folded to the head's dW / db."""
    stream_here = _stream_form()
    env = dict(os.environ, RSLRL_VALUE_HEAD_STREAM="0" if stream_here else "1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", __file__,
                        "-k", "test_value_head_matches_separate_launches"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
