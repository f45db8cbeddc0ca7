"""Fused fp32 MFMA MLP (networks/fused_mlp.py, csrc/mlp_gemm.hip) vs the same nn.Sequential evaluated
layer by layer by torch (hipBLASLt + ATen ELU).  Tolerance 1e-5 relative to each tensor's max: the MFMA
k-order differs from hipBLASLt's at fp32 epsilon."""

import pytest
import torch

from rsl_rl_amd import _lib
from rsl_rl_amd.networks import MLP
from rsl_rl_amd.networks import fused_mlp
from rsl_rl_amd.networks.fused_mlp import bimage, fusable_structure, linear_dgrad_elu, linear_fwd

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _close(a, b, tol=TOL):
    assert (a - b).abs().max().item() <= tol * b.abs().max().item() + 1e-12, (a - b).abs().max().item()


@pytest.fixture(params=["x6", "f32", "h3"])
def gemm_mode(request):
    prev = fused_mlp.set_gemm_mode(fused_mlp._MODE_NAMES[request.param])
    yield request.param
    fused_mlp.set_gemm_mode(prev)


def _reference(mlp, x):
    y = x
    for layer in mlp:
        y = layer(y)
    return y


@pytest.mark.parametrize("M,K,N,elu", [(393216, 256, 256, True), (65536, 48, 256, True), (1000, 16, 64, False),
                                       (777, 48, 48, True), (129, 256, 256, True), (1, 4, 8, True)])
def test_linear_fwd(M, K, N, elu, gemm_mode, cuda_device):
    torch.manual_seed(M)
    x = torch.randn(M, K, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / K ** 0.5
    b = torch.randn(N, device=cuda_device)
    ref = torch.nn.functional.linear(x, w, b)
    if elu:
        ref = torch.nn.functional.elu(ref)
    _close(linear_fwd(x, w, b, elu, bimage(w, False) if gemm_mode != "f32" else None), ref)


@pytest.mark.parametrize("M,N,K", [(393216, 256, 256), (5000, 12, 256), (1000, 64, 64), (300, 48, 48)])
def test_linear_dgrad_elu(M, N, K, gemm_mode, cuda_device):
    torch.manual_seed(N + K)
    dz = torch.randn(M, N, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / N ** 0.5
    h = torch.nn.functional.elu(torch.randn(M, K, device=cuda_device))
    out, db = linear_dgrad_elu(dz, w, h, bimage(w, True) if gemm_mode != "f32" else None)
    ref = dz.mm(w)
    ref = torch.where(h > 0, ref, ref * (h + 1))
    _close(out, ref)
    _close(db, ref.double().sum(0).float(), 1e-4)


@pytest.mark.parametrize("din,dout,hidden,M", [(48, 12, [256, 256, 256], 393216), (48, 1, [256, 256, 256], 65536),
                                               (16, 4, [64, 64], 2048), (48, [2, 12], [256, 256, 256], 5000),
                                               (48, 1, [-1], 3001)])
def test_mlp_forward_backward(din, dout, hidden, M, gemm_mode, cuda_device):
    torch.manual_seed(7)
    mlp = MLP(din, dout, hidden, "elu").to(cuda_device)
    assert mlp._fused and fusable_structure(mlp)
    x = torch.randn(M, din, device=cuda_device)
    y = mlp(x)
    g = torch.randn_like(y)
    y.backward(g)
    ours = [p.grad.clone() for p in mlp.parameters()]
    mlp.zero_grad()
    ref = _reference(mlp, x)
    _close(y, ref)
    ref.backward(g)
    for (name, p), a in zip(mlp.named_parameters(), ours):
        _close(a, p.grad, 2e-5 if "bias" in name else TOL)
    with torch.inference_mode():
        _close(mlp(x), ref.detach())


def test_input_gradient(gemm_mode, cuda_device):
    torch.manual_seed(3)
    mlp = MLP(48, 12, [256, 256], "elu").to(cuda_device)
    x = torch.randn(4096, 48, device=cuda_device, requires_grad=True)
    mlp(x).square().sum().backward()
    gx = x.grad.clone()
    x.grad = None
    _reference(mlp, x).square().sum().backward()
    _close(gx, x.grad)


def test_unfusable_structures_fall_back_to_layers():
    assert not fusable_structure(MLP(48, 12, [256], "relu"))
    assert not fusable_structure(MLP(50, 12, [256], "elu"))  # in_features % 4
    assert not fusable_structure(MLP(48, 12, [512], "elu"))  # width > 256



@pytest.mark.parametrize("kind", ["fwd", "dgrad"])
@pytest.mark.parametrize("M,K,N", [(65536, 256, 256), (65536, 48, 256), (4096, 256, 12)])
def test_x6_error_matches_fp32(kind, M, K, N, cuda_device):
    """The split-bf16 x6 GEMM is an fp32-class GEMM: against an fp64 evaluation its RMS error is within 2x
    of torch's fp32 GEMM (hipBLASLt) on the same data, i.e. at most one bit off (measured 0.8x on the plain
    GEMM, 1.5x after ELU on a 12-wide output), its max error within 3x (max over a few 10^4 outputs is
    noisy), its mean (bias) small against its RMS, and it is far below a bf16 GEMM's.
    The bf16 MFMA sums each 16-product block with alignment to its largest product, a slightly negative-
    biased rounding (scripts/experiments/mfma_bf16_accum.hip); measured bias ~0.06 RMS."""
    torch.manual_seed(K * N)
    F = torch.nn.functional
    if kind == "fwd":
        x = torch.randn(M, K, device=cuda_device)
        w = torch.randn(N, K, device=cuda_device) / K ** 0.5
        b = torch.randn(N, device=cuda_device)
        ref = F.linear(x.double(), w.double(), b.double())
        ref = torch.where(ref > 0, ref, torch.expm1(ref))
        ours = linear_fwd(x, w, b, True, bimage(w, False))
        torch_fp32 = F.elu(F.linear(x, w, b))
        bf16 = F.elu(F.linear(x.bfloat16(), w.bfloat16(), b.bfloat16()).float())
    else:
        if N % 4:
            pytest.skip("dgrad reduction width must be 4-aligned")
        dz = torch.randn(M, K, device=cuda_device)
        w = torch.randn(K, N, device=cuda_device) / K ** 0.5
        h = F.elu(torch.randn(M, N, device=cuda_device))
        d = dz.double().mm(w.double())
        ref = torch.where(h > 0, d, d * (h.double() + 1))
        ours = linear_dgrad_elu(dz, w, h, bimage(w, True))[0]
        d32 = dz.mm(w)
        torch_fp32 = torch.where(h > 0, d32, d32 * (h + 1))
        d16 = dz.bfloat16().mm(w.bfloat16()).float()
        bf16 = torch.where(h > 0, d16, d16 * (h + 1))
    def err(a):
        d = a.double() - ref
        return d.abs().max().item(), d.square().mean().sqrt().item(), d.mean().item()

    (m_ours, r_ours, b_ours), (m_fp32, r_fp32, _), (m_bf16, r_bf16, _) = err(ours), err(torch_fp32), err(bf16)
    assert r_ours <= 2.0 * r_fp32, (r_ours, r_fp32)
    assert m_ours <= 3.0 * m_fp32, (m_ours, m_fp32)
    assert abs(b_ours) <= 0.25 * r_ours, (b_ours, r_ours)
    assert r_ours * 100 < r_bf16 and m_ours * 30 < m_bf16, (r_ours, r_bf16, m_ours, m_bf16)


def test_weights_updated_in_place_are_seen(gemm_mode, cuda_device):
    """Fused Adam updates parameters without moving their version counter: the next forward must still use
    the new weights (B images are rebuilt per call outside frozen_weights())."""
    torch.manual_seed(11)
    mlp = MLP(48, 12, [256, 256], "elu").to(cuda_device)
    opt = torch.optim.Adam(mlp.parameters(), lr=1e-2, fused=True)
    x = torch.randn(512, 48, device=cuda_device)
    for _ in range(3):
        y = mlp(x)
        ref = _reference(mlp, x)
        _close(y, ref)
        opt.zero_grad()
        y.square().mean().backward()
        opt.step()
    with torch.inference_mode():
        _close(mlp(x), _reference(mlp, x))


def test_frozen_weights_scope_reuses_images(cuda_device):
    torch.manual_seed(12)
    mlp = MLP(48, 12, [256, 256], "elu").to(cuda_device)
    x = torch.randn(1000, 48, device=cuda_device)
    with torch.inference_mode(), fused_mlp.frozen_weights():
        a = mlp(x)
        # two hidden-layer images (+ the output-layer image when the output layer is fused into the last
        # hidden layer's forward)
        assert len(fused_mlp._bimage_cache) == 2 + int(fused_mlp._fuse_out_fwd([m.weight for m in mlp
                                                                                 if isinstance(m, torch.nn.Linear)]))
        b = mlp(x)
    assert len(fused_mlp._bimage_cache) == 0
    assert torch.equal(a, b)
    with torch.no_grad():
        _close(a, _reference(mlp, x))


@pytest.mark.parametrize("M,N,K", [(393216, 256, 256), (393216, 256, 48), (393216, 48, 256), (1000, 64, 256),
                                   (777, 40, 200), (5000, 12, 256), (3001, 4, 256),
                                   (100, 256, 256), (16, 32, 64), (70000, 64, 128)])
def test_linear_wgrad(M, N, K, cuda_device):
    """dW = dz^T x on the x6 weight-gradient kernel: fp32-class error against fp64 (RMS within 2x of torch's
    fp32 GEMM), deterministic (two calls bit-identical)."""
    torch.manual_seed(M + N + K)
    dz = torch.randn(M, N, device=cuda_device)
    x = torch.nn.functional.elu(torch.randn(M, K, device=cuda_device))
    ref = dz.double().t().mm(x.double())
    ours = fused_mlp.linear_wgrad(dz, x)
    assert torch.equal(ours, fused_mlp.linear_wgrad(dz, x))
    t32 = dz.t().mm(x)
    rms = lambda a: (a.double() - ref).square().mean().sqrt().item()  # noqa: E731
    assert rms(ours) <= 2.0 * rms(t32) + 1e-12, (rms(ours), rms(t32))
    _close(ours, ref.float(), 1e-5)


@pytest.mark.parametrize("M,N,K", [(393216, 12, 256), (5000, 4, 256), (3001, 16, 64), (128, 8, 48), (393216, 1, 256),
                                   (3001, 3, 256), (1000, 5, 48)])
def test_linear_dgrad_elu_wgrad(M, N, K, cuda_device):
    """Fused output-layer backward (one x6 launch): dz_prev and the bias grad as linear_dgrad_elu, and the
    layer's weight gradient dz^T h, vs fp64 (fp32-class: 2e-5 of the max, the sum runs over M rows)."""
    torch.manual_seed(M + N)
    dz = torch.randn(M, N, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / N ** 0.5
    h = torch.nn.functional.elu(torch.randn(M, K, device=cuda_device))
    out, db, dw, db_out = fused_mlp.linear_dgrad_elu_wgrad(dz, w, h, bimage(w, True))
    d = dz.double().mm(w.double())
    ref = torch.where(h > 0, d, d * (h.double() + 1))
    _close(out, ref.float())
    _close(db, ref.sum(0).float(), 1e-4)
    _close(dw, dz.double().t().mm(h.double()).float(), 2e-5)
    _close(db_out, dz.double().sum(0).float(), 1e-5)  # this layer's own bias gradient (column sums of dz)
    out2, db2, dw2, db_out2 = fused_mlp.linear_dgrad_elu_wgrad(dz, w, h, bimage(w, True))
    assert torch.equal(dw, dw2) and torch.equal(db, db2) and torch.equal(db_out, db_out2)  # deterministic
    if N % 4:  # rows of Nred floats read as they are == the zero-padded operand (the round-2 layout), bitwise
        pad = (-N) % 4
        wp = torch.nn.functional.pad(w, (0, 0, 0, pad))
        out3, db3, dw3, db_out3 = fused_mlp.linear_dgrad_elu_wgrad(torch.nn.functional.pad(dz, (0, pad)), wp, h,
                                                                  bimage(wp, True))
        assert torch.equal(out, out3) and torch.equal(db, db3)
        assert torch.equal(dw, dw3[:N]) and torch.equal(db_out, db_out3[:N])


@pytest.mark.parametrize("S,NK", [(1, 4), (7, 100), (256, 65536), (3072, 3072), (3072, 1024), (129, 20)])
def test_fold_partials(S, NK, cuda_device):
    """rslrl_fold_partials (one- and two-stage) vs an fp64 sum; bitwise repeatable."""
    L = _lib.lib()
    torch.manual_seed(S + NK)
    part = torch.randn(S, NK, device=cuda_device)
    nbytes = L.rslrl_fold_partials_workspace_bytes(S, NK)
    ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=cuda_device)
    outs = []
    for _ in range(2):
        out = torch.empty(NK, device=cuda_device)
        _lib.check(L.rslrl_fold_partials(part.data_ptr(), S, NK, out.data_ptr(), ws.data_ptr(), nbytes,
                                         torch.cuda.current_stream().cuda_stream), "fold")
        outs.append(out)
    ref = part.double().sum(0)
    assert torch.allclose(outs[0].double(), ref, rtol=1e-6, atol=1e-6)
    assert torch.equal(outs[0], outs[1])


_X6S_CHECK = r"""
import torch
from rsl_rl_amd.networks import fused_mlp
from rsl_rl_amd.networks.fused_mlp import bimage, linear_fwd
fused_mlp.set_gemm_mode(fused_mlp.GEMM_X6)
torch.manual_seed(0)
dev = torch.device("cuda:0")
for M, K, N, elu in [(65536, 256, 256, True), (65536, 48, 256, False), (1000, 16, 64, True), (333, 256, 128, True)]:
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    y = linear_fwd(x, w, b, elu, bimage(w, False))
    z = x.double().mm(w.double().t()) + b.double()
    ref = torch.nn.functional.elu(z) if elu else z
    err = (y.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-6, (M, K, N, elu, err)
    assert torch.equal(y, linear_fwd(x, w, b, elu, bimage(w, False)))
print("ok")
"""


def test_x6_16x16_forward_opt_in(cuda_device):
    """The opt-in 16x16x32 paired-x6 forward kernel (RSLRL_X6_SHAPE=16, read once per process: run in a child
    process) vs fp64, full and ragged tiles, bitwise repeatable."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, RSLRL_X6_SHAPE="16")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _X6S_CHECK], env=env, cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("M,K,N,nout,store", [(393216, 256, 256, 12, True), (65536, 256, 256, 1, False),
                                              (1000, 64, 128, 7, True), (333, 48, 256, 32, True),
                                              (130, 256, 60, 3, False)])
def test_linear_fwd_out(M, K, N, nout, store, cuda_device):
    """Last hidden layer + output layer in one x6 launch: h = ELU(x W^T + b) (stored or not) and
    y = h W_out^T + b_out vs fp64 (fp32-class: 1e-5 of the max), bitwise repeatable."""
    torch.manual_seed(M + nout)
    x = torch.randn(M, K, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / K ** 0.5
    b = torch.randn(N, device=cuda_device) * 0.1
    wo = torch.randn(nout, N, device=cuda_device) / N ** 0.5
    bo = torch.randn(nout, device=cuda_device)
    img, oimg = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT)])
    h, y = fused_mlp.linear_fwd_out(x, w, b, img, wo, bo, oimg, store_h=store)
    href = torch.nn.functional.elu(x.double().mm(w.double().t()) + b.double())
    yref = href.mm(wo.double().t()) + bo.double()
    _close(y, yref.float())
    if store:
        _close(h, href.float())
    else:
        assert h is None
    h2, y2 = fused_mlp.linear_fwd_out(x, w, b, img, wo, bo, oimg, store_h=store)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("S,R,C,E,out_len", [(37, 48, 256, 256, None), (256, 48, 256, 256, None),
                                              (3072, 0, 0, 260, 257), (7, 0, 0, 100, 98)])
def test_fold_partials_mapped(S, R, C, E, out_len, cuda_device):
    """rslrl_fold_partials_ex: the leading R x C block written transposed and only out_len sums written -- bitwise
    the identity fold's values at their mapped places, nothing past out_len touched."""
    L = _lib.lib()
    torch.manual_seed(S + E)
    NK = R * C + E
    out_len = NK if out_len is None else out_len
    part = torch.randn(S, NK, device=cuda_device)
    nbytes = L.rslrl_fold_partials_workspace_bytes(S, NK)
    ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=cuda_device)
    ident = torch.empty(NK, device=cuda_device)
    _lib.check(L.rslrl_fold_partials(part.data_ptr(), S, NK, ident.data_ptr(), ws.data_ptr(), nbytes,
                                     torch.cuda.current_stream().cuda_stream), "fold")
    buf = torch.full((out_len + 3,), float("nan"), device=cuda_device)
    dst = buf[1:]  # 4-byte aligned only
    _lib.check(L.rslrl_fold_partials_ex(part.data_ptr(), S, NK, dst.data_ptr(), out_len, R, C, ws.data_ptr(), nbytes,
                                        torch.cuda.current_stream().cuda_stream), "fold_ex")
    torch.cuda.synchronize()
    if R:
        assert torch.equal(dst[: R * C].view(C, R), ident[: R * C].view(R, C).t())
    assert torch.equal(dst[R * C: out_len], ident[R * C: out_len])
    assert torch.isnan(buf[0]) and torch.isnan(buf[out_len + 1:]).all()


def test_fold_partials_batch(cuda_device):
    """rslrl_fold_partials_batch: several folds (wide and narrow, mapped and not) in one launch -- each bitwise the
    one-pass wide fold of its job and within fp32 rounding of an fp64 sum."""
    L = _lib.lib()
    torch.manual_seed(3)
    specs = [(256, 48 * 256 + 256, 48, 256), (128, 65536 + 256, 0, 0), (3072, 3084, 0, 0), (768, 260, 0, 0), (5, 8, 0, 0)]
    parts, outs, jobs = [], [], []
    for S, NK, tr, tc in specs:
        part = torch.randn(S, NK, device=cuda_device)
        out_len = NK - 3 if NK == 260 else NK
        out = torch.full((out_len,), float("nan"), device=cuda_device)
        parts.append(part)
        outs.append(out)
        jobs.append(_lib.FoldJob(part.data_ptr(), S, NK, out.data_ptr(), out_len, tr, tc))
    arr = (_lib.FoldJob * len(jobs))(*jobs)
    nbytes = L.rslrl_fold_partials_batch_workspace_bytes(arr, len(jobs))
    ws = torch.zeros(max(nbytes, 256) // 8 + 32, dtype=torch.float64, device=cuda_device)
    for _ in range(2):  # the second call reuses the workspace: its counters must have been left zero
        for o in outs:
            o.fill_(float("nan"))
        _lib.check(L.rslrl_fold_partials_batch(arr, len(jobs), ws.data_ptr(), ws.numel() * 8,
                                               torch.cuda.current_stream().cuda_stream), "batch")
    torch.cuda.synchronize()
    assert nbytes > 256  # the 3072-slice narrow jobs are grouped
    for (S, NK, tr, tc), part, out in zip(specs, parts, outs):
        ref = part.double().sum(0)
        if tr:
            ref = torch.cat([ref[: tr * tc].view(tr, tc).t().reshape(-1), ref[tr * tc:]])
        ref = ref[: out.numel()]
        assert not torch.isnan(out).any()
        assert ((out.double() - ref).abs() <= 1e-6 * ref.abs() + 1e-6).all()
