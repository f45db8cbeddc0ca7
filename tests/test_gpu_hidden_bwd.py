"""The fused backward of a square hidden layer (rslrl_hidden_bwd_pair, csrc/mlp_bwd_fused.hip: the input gradient and
the weight + bias gradients of Linear(256, 256) + ELU from one read of dz and h) against the separate launches it
replaces -- linear_dgrad_elu_pair (the input gradient: bit-identical) and linear_wgrad_pair(bias_side=1) (the weight
and bias gradients: the same sums over the rows in another order, so within fp32 accumulation error) -- and against an
fp64 reference of dz^T h.  Reference arithmetic: the autograd backward of rsl_rl/networks/mlp.py:106-114's layers
(ppo.py:367)."""

import numpy as np
import pytest
import torch

from rsl_rl_amd import _lib
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu
W = 256


def _problem(M, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    dz = torch.randn(M, W, device=dev, generator=g) * 0.01
    h = torch.nn.functional.elu(torch.randn(M, W, device=dev, generator=g))
    w = torch.randn(W, W, device=dev, generator=g) / 16
    return dz, h, w


def _close(a, b, rtol):
    scale = float(b.abs().max()) + 1e-30
    return float((a - b).abs().max()) <= rtol * scale


@pytest.mark.parametrize("M", [64, 4096, 98304, 393216])
def test_hidden_bwd_pair_matches_separate_launches(M, cuda_device):
    dev = cuda_device
    p = [_problem(M, dev, 11 + M), _problem(M, dev, 12 + M)]
    dzs, hs = [q[0] for q in p], [q[1] for q in p]
    imgs = fused_mlp.bimages([(q[2], True) for q in p])
    assert fused_mlp.hidden_bwd_ok(dzs, hs)
    got = fused_mlp.hidden_bwd_pair(dzs, hs, imgs)
    ref_dz, _ = fused_mlp.linear_dgrad_elu_pair(dzs, hs, imgs, _lib.ARITH_X6)
    ref_w = fused_mlp.linear_wgrad_pair(dzs, hs, bias_side=1)
    torch.cuda.synchronize()
    for i in range(2):
        dzp, dw, db = got[i]
        assert torch.equal(dzp, ref_dz[i]), i  # the same products in the same order: the same bits
        assert _close(dw, ref_w[i][0], 1e-5), (i, float((dw - ref_w[i][0]).abs().max()))
        assert _close(db, ref_w[i][1], 1e-5), i
        # against fp64: the error of an fp32-class GEMM over M rows
        dw64 = dzs[i].double().t() @ hs[i].double()
        db64 = dzs[i].double().sum(0)
        err = float((dw.double() - dw64).abs().max())
        err_ref = float((ref_w[i][0].double() - dw64).abs().max())
        assert err <= 3 * err_ref + 1e-12 * float(dw64.abs().max()), (err, err_ref)
        assert _close(db.double(), db64, 2e-6)
    # deterministic: a second launch gives the same bits
    again = fused_mlp.hidden_bwd_pair(dzs, hs, imgs)
    torch.cuda.synchronize()
    for a, b in zip(got, again):
        for u, v in zip(a, b):
            assert torch.equal(u, v)


def test_hidden_bwd_single_problem_and_declines(cuda_device):
    dev = cuda_device
    dz, h, w = _problem(8192, dev, 3)
    img = fused_mlp.bimages([(w, True)])
    one = fused_mlp.hidden_bwd_pair([dz], [h], img)[0]
    pair = fused_mlp.hidden_bwd_pair([dz, dz], [h, h], [img[0], img[0]])
    torch.cuda.synchronize()
    for u, v in zip(one, pair[0]):
        assert torch.equal(u, v)
    # rows not a multiple of 64: the C ABI launches nothing
    assert not fused_mlp.hidden_bwd_ok([dz[:1000]], [h[:1000]])
    L = _lib.lib()
    prob = _lib.HiddenBwdProblem(dz.data_ptr(), h.data_ptr(), img[0].data_ptr(), dz.data_ptr(), dz.data_ptr())
    assert L.rslrl_hidden_bwd_pair(prob, None, 1000, W, None) == -3  # RSLRL_E_UNSUPPORTED
    assert L.rslrl_hidden_bwd_pair(prob, None, 1024, 128, None) == -1  # only the 256-wide layer


def test_update_with_hidden_bwd(cuda_device, monkeypatch):
    """PPO.update() with the fused hidden-layer backward and with the separate launches on one storage: the same
    learning-rate trace, loss statistics rtol 1e-4, parameters within fp32 accumulation-order noise."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    dev = cuda_device
    T, N, O, A = 8, 2048, 48, 12
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    rng = np.random.default_rng(9)
    data = {k: rng.standard_normal(s).astype(np.float32) for k, s in
            (("obs", (T, N, O)), ("rewards", (T, N, 1)), ("values", (T, N, 1)), ("logp", (T, N, 1)),
             ("mu", (T, N, A)), ("actions", (T, N, A)), ("last", (N, O)))}
    results = []
    for use in (True, False):
        monkeypatch.setattr(fused_mlp, "_HIDDEN_BWD", use)
        calls = []
        real = fused_mlp.hidden_bwd_pair
        monkeypatch.setattr(fused_mlp, "hidden_bwd_pair", lambda *a, **k: calls.append(1) or real(*a, **k))
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
        assert len(calls) == (16 if use else 0)  # 8 mini-batches x the two square hidden layers
        results.append((loss, alg.learning_rate, {k: v.detach().clone() for k, v in pol.state_dict().items()}))
    (l1, lr1, p1), (l0, lr0, p0) = results
    assert lr1 == lr0
    for k in l0:
        assert np.isclose(l1[k], l0[k], rtol=1e-4, atol=1e-7), k
    for k in p0:
        assert torch.allclose(p1[k], p0[k], rtol=1e-4, atol=2e-6), k
