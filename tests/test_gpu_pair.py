"""rslrl_linear_gemm_pair (two same-shape forward problems in one launch: the rollout's actor and critic layers)
against two rslrl_linear_gemm calls -- bit-identical outputs and amaxes -- and ActorCritic.act_and_evaluate
against act() + evaluate() (ppo.py:155-156) with the same generator state."""

import pytest
import torch

from rsl_rl_amd import _lib
from rsl_rl_amd.modules import ActorCritic
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,arith", [(65536, 48, "x6"), (65536, 256, "h3"), (1000, 256, "h3"), (777, 48, "x6")])
def test_pair_matches_two_launches(M, K, arith, cuda_device):
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(3)
    N = 256
    xs = [torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g)) * s for s in (1.0, 37.0)]
    ws = [torch.randn(N, K, device=dev, generator=g) / K ** 0.5 for _ in range(2)]
    bs = [torch.randn(N, device=dev, generator=g) * 0.1 for _ in range(2)]
    h3 = arith == "h3"
    layout = _lib.BIMAGE_LAYOUT_H3 if h3 else _lib.BIMAGE_LAYOUT_GEMM
    imgs = fused_mlp.bimages([(w, False, layout) for w in ws])
    ar = _lib.ARITH_H3 if h3 else _lib.ARITH_X6
    x_amax = [x.abs().amax().reshape(1) if h3 else None for x in xs]
    ref = [fused_mlp.linear_fwd_ex(xs[i], bs[i], N, True, imgs[i], ar, x_amax[i], want_amax=True) for i in range(2)]
    ys, amaxes = fused_mlp.linear_fwd_pair(xs, bs, N, True, imgs, ar, x_amax, [True, True])
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(ys[i], ref[i][0])
        assert torch.equal(amaxes[i], ref[i][1])
        assert float(amaxes[i]) == float(ys[i].abs().max())


@pytest.mark.parametrize("K", [256, 48])
@pytest.mark.parametrize("M", [393216, 212992, 65536, 16384 + 128, 4096, 384, 128, 1000])
def test_stream_forward_pair_matches_tiled_kernel(M, K, cuda_device):
    """The x6 forward pair without amax of the square hidden layers (the update's and the rollout's path) runs on the
    streaming kernel (mlp_fwd_stream.hip) when M is a multiple of 128 of >= 1536 or <= 128 tiles (65,536 and 16,512
    rows stay on the tiled pair): its H must equal the tiled kernel's (the single-problem launch) bit for bit --
    slices of 1, 13 and 24 tiles (odd and even counts: the two accumulator sets alternate by tile), the last slice
    shorter, and a ragged M that stays on the tiled pair kernel.  K = 48 (the first
    layer) takes the streaming kernel only with RSLRL_FWD_STREAM=48 (measured bit-exact there too at every M below,
    profiles/r5_fs_ab.json); by default it checks the tiled pair against the single launch."""
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(M + K)
    N = 256
    xs = [torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g)) * s for s in (1.0, 9.0)]
    ws = [torch.randn(N, K, device=dev, generator=g) / K ** 0.5 for _ in range(2)]
    bs = [torch.randn(N, device=dev, generator=g) * 0.1 for _ in range(2)]
    imgs = fused_mlp.bimages([(w, False, _lib.BIMAGE_LAYOUT_GEMM) for w in ws])
    ref = [fused_mlp.linear_fwd_ex(xs[i], bs[i], N, True, imgs[i], _lib.ARITH_X6, None, want_amax=False)[0]
           for i in range(2)]
    ys, _ = fused_mlp.linear_fwd_pair(xs, bs, N, True, imgs, _lib.ARITH_X6, [None, None], [False, False])
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(ys[i], ref[i]), (i, float((ys[i] - ref[i]).abs().max()))
    # fp32 sanity against torch (x6 is fp32-faithful)
    y64 = torch.nn.functional.elu(xs[1].double() @ ws[1].double().t() + bs[1].double())
    assert float((ys[1].double() - y64).abs().max()) <= 1e-5 * float(y64.abs().max())


def test_pair_rejects_mismatched_shapes(cuda_device):
    x = torch.randn(128, 48, device=cuda_device)
    w = torch.randn(256, 48, device=cuda_device)
    b = torch.zeros(256, device=cuda_device)
    img = fused_mlp.bimages([(w, False)])[0]
    y = torch.empty(128, 256, device=cuda_device)
    a0 = fused_mlp._gemm_args(_lib.LINEAR_FWD_ELU, _lib.ARITH_X6, x, None, 256, img, bias=b, c=y)
    a1 = fused_mlp._gemm_args(_lib.LINEAR_FWD_ELU, _lib.ARITH_X6, x[:64], None, 256, img, bias=b, c=y)
    import ctypes

    L = _lib.lib()
    assert L.rslrl_linear_gemm_pair(ctypes.byref(a0), ctypes.byref(a1), None) == -1  # RSLRL_E_INVALID_ARGUMENT
    a1 = fused_mlp._gemm_args(_lib.LINEAR_DGRAD_ELU, _lib.ARITH_X6, x, None, 256, img, bias=b, c=y)
    assert L.rslrl_linear_gemm_pair(ctypes.byref(a0), ctypes.byref(a1), None) == -3  # RSLRL_E_UNSUPPORTED


@pytest.mark.parametrize("critic_width,state_dependent_std", [(48, False), (48, True), (52, False)])
def test_act_and_evaluate_matches_two_calls(critic_width, state_dependent_std, cuda_device, monkeypatch):
    """Same obs width: every hidden layer but the fused output layer goes through the pair launch; another
    critic width: the pair does not qualify and the two forwards run.  (The layer-by-layer pair path: the one-launch
    rollout forward, taken by default where it applies, is tests/test_gpu_rollout_mlp.py's.)"""
    monkeypatch.setattr(fused_mlp, "_ROLLOUT_MLP", False)
    torch.manual_seed(0)
    obs = {"policy": torch.randn(4096, 48, device=cuda_device),
           "critic": torch.randn(4096, critic_width, device=cuda_device)}
    groups = {"policy": ["policy"], "critic": ["critic"]}
    pol = ActorCritic(obs, groups, 12, actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256],
                      actor_obs_normalization=True, critic_obs_normalization=True,
                      state_dependent_std=state_dependent_std).to(cuda_device)
    pol.update_normalization(obs)
    calls = []
    pair = fused_mlp.linear_fwd_pair
    monkeypatch.setattr(fused_mlp, "linear_fwd_pair", lambda *a, **k: (calls.append(1), pair(*a, **k))[1])
    with torch.inference_mode():
        torch.cuda.manual_seed(5)
        a_ref = pol.act(obs)
        mean_ref, std_ref = pol.action_mean.clone(), pol.action_std.clone()
        v_ref = pol.evaluate(obs)
        torch.cuda.manual_seed(5)
        a, v = pol.act_and_evaluate(obs)
    assert len(calls) == (2 if critic_width == 48 else 0)
    assert torch.equal(a, a_ref) and torch.equal(v, v_ref)
    assert torch.equal(pol.action_mean, mean_ref) and torch.equal(pol.action_std, std_ref)


@pytest.mark.parametrize("M", [1000, 16384, 65536])
def test_out_pair_matches_two_launches(M, cuda_device):
    """The two fused output layers (12 outputs on the MFMA epilogue, 1 on the VALU one) through the pair entry --
    one launch while the tiles fit one per CU (M <= 16384 here), two launches past that -- bit-identical to two
    linear_fwd_out_ex calls, full and partial tiles."""
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(5)
    K, N = 256, 256
    xs = [torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g)) for _ in range(2)]
    ws = [torch.randn(N, K, device=dev, generator=g) / 16 for _ in range(2)]
    bs = [torch.randn(N, device=dev, generator=g) * 0.1 for _ in range(2)]
    wo = [torch.randn(n, N, device=dev, generator=g) / 16 for n in (12, 1)]
    bo = [torch.randn(n, device=dev, generator=g) * 0.1 for n in (12, 1)]
    imgs = fused_mlp.bimages([(w, False) for w in ws] + [(w, False, _lib.BIMAGE_LAYOUT_OUT) for w in wo])
    for store_h in (False, True):
        ref = [fused_mlp.linear_fwd_out_ex(xs[i], bs[i], N, imgs[i], _lib.ARITH_X6, None, bo[i], imgs[2 + i],
                                           store_h=store_h) for i in range(2)]
        hs, ys = fused_mlp.linear_fwd_out_pair(xs, bs, N, imgs[:2], bo, imgs[2:], store_h=store_h)
        torch.cuda.synchronize()
        for i in range(2):
            assert torch.equal(ys[i], ref[i][1])
            if store_h:
                assert torch.equal(hs[i], ref[i][0])


@pytest.mark.parametrize("M,w4", [(777, None), (98304, None), (262144, None), (98304, "1")])
def test_dgrad_pair_matches_two_launches(M, w4, cuda_device, monkeypatch):
    """Two hidden-layer input gradients (dz W) * ELU'(h) in one launch, bit-identical to two launches -- including the
    4-wave 128 x 64 layout ("w4": the default at >= 2048 tiles per problem, forced with RSLRL_W4=1)."""
    if w4 is not None:
        monkeypatch.setenv("RSLRL_W4", w4)
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(6)
    dzs = [torch.randn(M, 256, device=dev, generator=g) for _ in range(2)]
    hs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev, generator=g)) for _ in range(2)]
    ws = [torch.randn(256, 256, device=dev, generator=g) / 16 for _ in range(2)]
    imgs = [fused_mlp.bimage(w, True) for w in ws]
    ref = [fused_mlp.linear_dgrad_elu_ex(dzs[i], hs[i], imgs[i], _lib.ARITH_X6, want_db=False)[0] for i in range(2)]
    outs, _ = fused_mlp.linear_dgrad_elu_pair(dzs, hs, imgs, _lib.ARITH_X6)
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(outs[i], ref[i])


def test_w4_forward_pair_matches(cuda_device, monkeypatch):
    """The opt-in w4 layout on the hidden forward (RSLRL_W4=1) gives the default launch's bits."""
    dev = cuda_device
    g = torch.Generator(device=dev).manual_seed(7)
    M = 65536
    xs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev, generator=g)) for _ in range(2)]
    ws = [torch.randn(256, 256, device=dev, generator=g) / 16 for _ in range(2)]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(2)]
    imgs = fused_mlp.bimages([(w, False) for w in ws])
    monkeypatch.setenv("RSLRL_W4", "0")
    ref, _ = fused_mlp.linear_fwd_pair(xs, bs, 256, True, imgs, _lib.ARITH_X6, [None, None], [False, False])
    monkeypatch.setenv("RSLRL_W4", "1")
    ys, _ = fused_mlp.linear_fwd_pair(xs, bs, 256, True, imgs, _lib.ARITH_X6, [None, None], [False, False])
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(ys[i], ref[i])
