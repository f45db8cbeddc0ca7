"""rslrl_rollout_mlp_pair (the rollout's actor and critic forward, every layer in one launch: rollout_mlp.hip) against
the layer-by-layer launches of fused_mlp_forward_pair (rslrl_linear_gemm_pair per hidden layer, then the fused last
hidden + output layer) -- bit-identical outputs -- and against fp64 torch (x6 is fp32-faithful); the shapes it declines
run the layer-by-layer path.  The reference computation is policy.act / policy.evaluate's MLPs (ppo.py:155-156,
rsl_rl/networks/mlp.py:106-114)."""

import ctypes

import pytest
import torch
import torch.nn as nn

from rsl_rl_amd import _lib
from rsl_rl_amd.modules import ActorCritic
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu


def _mlp(k0, hidden, nout, dev, g):
    layers, d = [], k0
    for _ in range(hidden):
        lin = nn.Linear(d, 256)
        layers += [lin, nn.ELU()]
        d = 256
    layers.append(nn.Linear(256, nout))
    m = nn.Sequential(*layers).to(dev)
    with torch.no_grad():
        for p in m.parameters():  # weights of the scale training reaches, biases that push ELU across both branches
            p.copy_(torch.randn(p.shape, device=dev, generator=g) * (0.3 if p.dim() == 1 else 1.2 / p.shape[-1] ** 0.5))
    return m


def _both(ma, xa, mb, xb, monkeypatch):
    """(one-launch result, layer-by-layer result, one-launch call count)"""
    n0 = fused_mlp.rollout_mlp_launches
    with torch.inference_mode():
        one = fused_mlp.fused_mlp_forward_pair(ma, xa, mb, xb)
        n1 = fused_mlp.rollout_mlp_launches - n0
        monkeypatch.setattr(fused_mlp, "_ROLLOUT_MLP", False)
        ref = fused_mlp.fused_mlp_forward_pair(ma, xa, mb, xb)
        monkeypatch.setattr(fused_mlp, "_ROLLOUT_MLP", True)
    torch.cuda.synchronize()
    return one, ref, n1


@pytest.mark.parametrize("M,k0,hidden,nouts", [
    (16384, 48, 3, (12, 1)),    # C4's rollout share per GPU at 8 GPUs (C3's MLPs)
    (65536, 48, 3, (12, 1)),    # C3's rollout
    (64, 48, 3, (12, 1)),       # one tile per problem
    (4160, 48, 3, (12, 1)),     # 65 tiles: not a multiple of the layer-by-layer kernels' 128 rows
    (8192, 16, 2, (4, 3)),      # <= 4 outputs on both: the fp32 fma output layer twice
    (8192, 64, 4, (16, 2)),     # the widest input, output and depth covered
    (2048, 32, 3, (7, 1)),      # an odd output width on the MFMA output layer
])
def test_rollout_mlp_matches_layer_by_layer(M, k0, hidden, nouts, cuda_device, monkeypatch):
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(M + k0 + hidden)
    ma, mb = _mlp(k0, hidden, nouts[0], dev, g), _mlp(k0, hidden, nouts[1], dev, g)
    xa = torch.randn(M, k0, device=dev, generator=g)
    xb = torch.randn(M, k0, device=dev, generator=g) * 3.0
    one, ref, n = _both(ma, xa, mb, xb, monkeypatch)
    assert n == 1
    for i in range(2):
        assert one[i].shape == ref[i].shape
        assert torch.equal(one[i], ref[i]), (i, float((one[i] - ref[i]).abs().max()))
    for m, x, y in ((ma, xa, one[0]), (mb, xb, one[1])):  # fp32-faithful against fp64
        y64 = m.double()(x.double())
        m.float()
        assert float((y.double() - y64).abs().max()) <= 2e-5 * max(1.0, float(y64.abs().max()))


@pytest.mark.parametrize("M,k0,hidden,nouts", [
    (1000, 48, 3, (12, 1)),     # not a multiple of 64 rows
    (4096, 52, 3, (12, 1)),     # input width not a multiple of 16
    (4096, 48, 1, (12, 1)),     # one hidden layer
    (4096, 48, 3, (24, 1)),     # a state-dependent std head: 24 outputs
])
def test_rollout_mlp_declines_to_layer_by_layer(M, k0, hidden, nouts, cuda_device, monkeypatch):
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(7)
    ma, mb = _mlp(k0, hidden, nouts[0], dev, g), _mlp(k0, hidden, nouts[1], dev, g)
    xa, xb = torch.randn(M, k0, device=dev, generator=g), torch.randn(M, k0, device=dev, generator=g)
    one, ref, n = _both(ma, xa, mb, xb, monkeypatch)
    assert n == 0
    for i in range(2):
        assert torch.equal(one[i], ref[i])


def test_rollout_mlp_c_abi_rejects(cuda_device):
    """Unsupported shapes return RSLRL_E_UNSUPPORTED with nothing launched; M = 0 is a no-op."""
    L = _lib.lib()
    dev = cuda_device
    x = torch.zeros(128, 48, device=dev)
    y = torch.full((128, 12), 7.0, device=dev)
    a = _lib.RolloutMlp()
    a.x, a.k0, a.hidden, a.nout, a.y = x.data_ptr(), 48, 3, 12, y.data_ptr()
    for M, k0, hidden, nout in ((100, 48, 3, 12), (128, 40, 3, 12), (128, 48, 5, 12), (128, 48, 3, 17)):
        b = _lib.RolloutMlp.from_buffer_copy(a)
        b.k0, b.hidden, b.nout = k0, hidden, nout
        assert L.rslrl_rollout_mlp_pair(ctypes.byref(b), ctypes.byref(b), M, None) == _lib.E_UNSUPPORTED
    assert L.rslrl_rollout_mlp_pair(ctypes.byref(a), ctypes.byref(a), 0, None) == 0
    torch.cuda.synchronize()
    assert bool((y == 7.0).all())


def test_act_and_evaluate_takes_one_launch(cuda_device):
    """ActorCritic.act_and_evaluate (the rollout step, ppo.py:155-156) on C3's networks: one rollout_mlp launch per
    step, and the actions / values / distribution of act() + evaluate() bit for bit."""
    torch.manual_seed(0)
    obs = {"policy": torch.randn(8192, 48, device=cuda_device)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = ActorCritic(obs, groups, 12, actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256],
                      actor_obs_normalization=True, critic_obs_normalization=True).to(cuda_device)
    pol.update_normalization(obs)
    with torch.inference_mode():
        torch.cuda.manual_seed(5)
        a_ref = pol.act(obs)
        mean_ref = pol.action_mean.clone()
        v_ref = pol.evaluate(obs)
        n0 = fused_mlp.rollout_mlp_launches
        torch.cuda.manual_seed(5)
        a, v = pol.act_and_evaluate(obs)
        assert fused_mlp.rollout_mlp_launches == n0 + 1
    assert torch.equal(a, a_ref) and torch.equal(v, v_ref) and torch.equal(pol.action_mean, mean_ref)


@pytest.mark.parametrize("M,k0,hidden,nout", [
    (16384, 48, 3, 1),     # compute_returns' last values at the 16,384-env share (C3's critic)
    (4160, 48, 3, 12),     # 65 tiles, the actor (act_inference)
    (2048, 32, 2, 7),
])
def test_rollout_mlp_single_network_matches_layer_by_layer(M, k0, hidden, nout, cuda_device, monkeypatch):
    """One network through the one-launch kernel (a1 = NULL: fused_mlp_forward, i.e. policy.evaluate / act_inference)
    against its layer-by-layer launches, bit for bit."""
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(M + nout)
    m = _mlp(k0, hidden, nout, dev, g)
    x = torch.randn(M, k0, device=dev, generator=g)
    with torch.inference_mode():
        n0 = fused_mlp.rollout_mlp_launches
        one = fused_mlp.fused_mlp_forward(m, x)
        assert fused_mlp.rollout_mlp_launches == n0 + 1
        monkeypatch.setattr(fused_mlp, "_ROLLOUT_MLP", False)
        ref = fused_mlp.fused_mlp_forward(m, x)
    assert torch.equal(one, ref), float((one - ref).abs().max())


def test_rollout_mlp_sample_matches_normal_affine(cuda_device):
    """The Normal sample applied in the one-launch forward (eps <- eps * std + mu) against rslrl_normal_affine on the
    kernel's own mu, bit for bit; the outputs are those of the sample-free launch; a scale the kernel does not take
    (per-row) declines before launching."""
    from rsl_rl_amd import kernels

    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(11)
    M = 16384
    ma, mb = _mlp(48, 3, 12, dev, g), _mlp(48, 3, 1, dev, g)
    xa, xb = torch.randn(M, 48, device=dev, generator=g), torch.randn(M, 48, device=dev, generator=g)
    std = torch.rand(12, device=dev, generator=g) + 0.2
    eps = torch.randn(M, 12, device=dev, generator=g)
    eps0 = eps.clone()
    with torch.inference_mode():
        ya, yb, sampled = fused_mlp.fused_mlp_forward_pair(ma, xa, mb, xb, sample=(eps, std))
        assert sampled
        ra, rb = fused_mlp.fused_mlp_forward_pair(ma, xa, mb, xb)
        ref = kernels.normal_affine_(eps0.clone(), std.expand(M, 12), ra)
        assert torch.equal(ya, ra) and torch.equal(yb, rb)
        assert torch.equal(eps, ref)
        assert torch.equal(ref, eps0 * std + ra)  # torch's mul_ then add_
        per_row = torch.rand(M, 12, device=dev, generator=g)
        e2 = eps0.clone()
        ya2, _, sampled2 = fused_mlp.fused_mlp_forward_pair(ma, xa, mb, xb, sample=(e2, per_row))
        assert not sampled2 and torch.equal(e2, eps0) and torch.equal(ya2, ra)


def test_rollout_mlp_c_abi_single_and_sample_arguments(cuda_device):
    """a1 = NULL is one problem (M = 0 still a no-op); a sample without its scale is an invalid argument."""
    L = _lib.lib()
    x = torch.zeros(128, 48, device=cuda_device)
    y = torch.full((128, 12), 7.0, device=cuda_device)
    a = _lib.RolloutMlp()
    a.x, a.k0, a.hidden, a.nout, a.y = x.data_ptr(), 48, 3, 12, y.data_ptr()
    assert L.rslrl_rollout_mlp_pair(ctypes.byref(a), None, 0, None) == 0
    assert L.rslrl_rollout_mlp_pair(None, ctypes.byref(a), 128, None) == _lib.E_INVALID_ARGUMENT
    a.out_image, a.out_bias = x.data_ptr(), x.data_ptr()  # past the null checks: the sample check decides
    a.sample = y.data_ptr()
    assert L.rslrl_rollout_mlp_pair(ctypes.byref(a), None, 128, None) == _lib.E_INVALID_ARGUMENT
    torch.cuda.synchronize()
    assert bool((y == 7.0).all())
