"""h3 arithmetic of the fused linear ops (csrc/mlp_gemm.hip, csrc/mlp_wgrad.hip via rslrl_linear_gemm /
rslrl_linear_wgrad_ex): operands scaled by a power of two from their producer's max |x| (amax), split into two
fp16 planes, three fp16 MFMA products, fp32 accumulation.

The bar is the one tests/test_gpu_fused_mlp.py sets for x6: an fp32-class GEMM against an fp64 evaluation of
the same op -- RMS error within 2x of torch's fp32 GEMM on the same data, max error within 3x, mean error
small against the RMS, far below a bf16 GEMM -- including operands whose magnitudes sit far outside fp16's
range (1e-9 gradients, 1e4 activations), which the scales bring back.  amax outputs are exact maxima."""

import pytest
import torch
import torch.nn.functional as F

from rsl_rl_amd import _lib
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu

H3 = _lib.ARITH_H3


def _img(w, transposed, layout=_lib.BIMAGE_LAYOUT_H3):
    return fused_mlp.bimages([(w, transposed, layout)])[0]


def _errs(a, ref):
    d = a.double() - ref
    return d.abs().max().item(), d.square().mean().sqrt().item(), d.mean().item()


def _fp32_class(ours, ref, torch_fp32, bf16=None, bias_vs_fp32=False):
    (m, r, b), (m32, r32, _) = _errs(ours, ref), _errs(torch_fp32, ref)
    assert r <= 2.0 * r32, (r, r32)
    assert m <= 3.0 * m32, (m, m32)
    # bias_vs_fp32 (long reductions): the MFMA aligns each block's sum to the accumulator and truncates, a
    # negative bias that grows with the number of accumulation steps (x6 measures -0.9 of its RMS on the
    # same weight gradients); it must stay small against torch's own fp32 error there
    assert abs(b) <= 0.25 * (r32 if bias_vs_fp32 else r) + 1e-300, (b, r, r32)
    if bf16 is not None:
        _, r16, _ = _errs(bf16, ref)
        assert r * 100 < r16, (r, r16)


def _amax(t):
    return t.abs().amax().reshape(1).float()


@pytest.mark.parametrize("M,K,N,scale", [(65536, 256, 256, 1.0), (65536, 256, 256, 1e-9), (65536, 256, 256, 1e4),
                                         (4097, 64, 64, 1.0), (777, 200, 40, 3e-3), (1, 4, 8, 1.0)])
def test_h3_fwd(M, K, N, scale, cuda_device):
    torch.manual_seed(M + K)
    x = F.elu(torch.randn(M, K, device=cuda_device)) * scale
    w = torch.randn(N, K, device=cuda_device) / K ** 0.5
    b = torch.randn(N, device=cuda_device) * scale
    y, amax = fused_mlp.linear_fwd_ex(x, b, N, True, _img(w, False), H3, _amax(x), want_amax=True)
    z = F.linear(x.double(), w.double(), b.double())
    ref = torch.where(z > 0, z, torch.expm1(z))
    if M >= 4096:
        _fp32_class(y, ref, F.elu(F.linear(x, w, b)), F.elu(F.linear(x.bfloat16(), w.bfloat16(),
                                                                      b.bfloat16()).float()))
    else:
        assert (y.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert amax.item() == y.abs().max().item()  # exact max of what was stored
    y2, _ = fused_mlp.linear_fwd_ex(x, b, N, True, _img(w, False), H3, _amax(x))
    assert torch.equal(y, y2)


@pytest.mark.parametrize("M,N,K,scale", [(65536, 256, 256, 1.0), (65536, 256, 256, 1e-8), (3001, 64, 128, 1e3),
                                         (129, 12, 256, 1.0)])
def test_h3_dgrad(M, N, K, scale, cuda_device):
    torch.manual_seed(N * K)
    dz = torch.randn(M, N, device=cuda_device) * scale
    w = torch.randn(N, K, device=cuda_device) / N ** 0.5
    h = F.elu(torch.randn(M, K, device=cuda_device))
    out, db, amax = fused_mlp.linear_dgrad_elu_ex(dz, h, _img(w, True), H3, _amax(dz), want_amax=True)
    d = dz.double().mm(w.double())
    ref = torch.where(h > 0, d, d * (h.double() + 1))
    d32 = dz.mm(w)
    t32 = torch.where(h > 0, d32, d32 * (h + 1))
    if M >= 4096:
        _fp32_class(out, ref, t32)
    else:
        assert (out.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert (db.double() - ref.sum(0)).abs().max().item() <= 1e-4 * ref.sum(0).abs().max().item()
    assert amax.item() == out.abs().max().item()


@pytest.mark.parametrize("M,N,K,sdz,sx", [(393216, 256, 256, 1e-7, 1.0), (65536, 256, 256, 1.0, 30.0),
                                          (70000, 64, 128, 1e-3, 1e-3), (1000, 256, 256, 1.0, 1.0)])
def test_h3_wgrad(M, N, K, sdz, sx, cuda_device):
    torch.manual_seed(M + N)
    dz = torch.randn(M, N, device=cuda_device) * sdz
    x = F.elu(torch.randn(M, K, device=cuda_device)) * sx
    ref = dz.double().t().mm(x.double())
    ours = fused_mlp.linear_wgrad(dz, x, H3, _amax(dz), _amax(x))
    assert torch.equal(ours, fused_mlp.linear_wgrad(dz, x, H3, _amax(dz), _amax(x)))  # deterministic
    _fp32_class(ours, ref, dz.t().mm(x), bias_vs_fp32=True)
    _, r_x6, _ = _errs(fused_mlp.linear_wgrad(dz, x), ref)
    assert _errs(ours, ref)[1] <= 1.1 * r_x6  # no worse than the x6 kernel (measured 0.5x)


@pytest.mark.parametrize("M,K,N,nout,store", [(393216, 256, 256, 12, True), (65536, 256, 256, 1, False),
                                              (1000, 64, 128, 7, True)])
def test_h3_fwd_out(M, K, N, nout, store, cuda_device):
    torch.manual_seed(M + nout)
    x = F.elu(torch.randn(M, K, device=cuda_device))
    w = torch.randn(N, K, device=cuda_device) / K ** 0.5
    b = torch.randn(N, device=cuda_device) * 0.1
    wo = torch.randn(nout, N, device=cuda_device) / N ** 0.5
    bo = torch.randn(nout, device=cuda_device)
    img, oimg = fused_mlp.bimages([(w, False, _lib.BIMAGE_LAYOUT_H3), (wo, False, _lib.BIMAGE_LAYOUT_OUT)])
    h, y = fused_mlp.linear_fwd_out_ex(x, b, N, img, H3, _amax(x), bo, oimg, store_h=store)
    href = F.elu(x.double().mm(w.double().t()) + b.double())
    yref = href.mm(wo.double().t()) + bo.double()
    assert (y.double() - yref).abs().max().item() <= 1e-5 * yref.abs().max().item()
    if store:
        _fp32_class(h, href, F.elu(F.linear(x, w, b)))
    else:
        assert h is None


def test_amax_workspace_left_zero(cuda_device):
    x = torch.randn(10000, 64, device=cuda_device)
    w = torch.randn(64, 64, device=cuda_device)
    b = torch.zeros(64, device=cuda_device)
    for _ in range(3):
        fused_mlp.linear_fwd_ex(x, b, 64, False, _img(w, False, _lib.BIMAGE_LAYOUT_GEMM), _lib.ARITH_X6,
                                want_amax=True)
    torch.cuda.synchronize()
    assert int(fused_mlp._amax_workspace(x.device).abs().sum().item()) == 0


def test_h3_mlp_training_step_matches_torch(cuda_device):
    """A C3-shaped actor MLP (48 -> 3x256 -> 12) in h3 mode: outputs and every parameter gradient vs torch's
    fp32 layers within 1e-5 of each tensor's max (the fused_mlp tests' tolerance), gradients scaled like
    PPO's (1 / B)."""
    from rsl_rl_amd.networks import MLP

    prev = fused_mlp.set_gemm_mode(fused_mlp.GEMM_H3)
    try:
        torch.manual_seed(5)
        mlp = MLP(48, 12, [256, 256, 256], "elu").to(cuda_device)
        x = torch.randn(65536, 48, device=cuda_device)
        y = mlp(x)
        g = torch.randn_like(y) / y.shape[0]
        y.backward(g)
        ours = [p.grad.clone() for p in mlp.parameters()]
        mlp.zero_grad()
        ref = x
        for layer in mlp:
            ref = layer(ref)
        ref.backward(g)
        assert (y - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
        for (name, p), a in zip(mlp.named_parameters(), ours):
            assert (a - p.grad).abs().max().item() <= 2e-5 * p.grad.abs().max().item(), name
    finally:
        fused_mlp.set_gemm_mode(prev)
