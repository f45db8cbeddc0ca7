"""Actor/critic MLP forward + backward on fused MFMA GEMMs.

For an `MLP` of Linear(+ELU) hidden blocks and a final Linear (rsl_rl/networks/mlp.py:59-114) this
autograd Function runs

    forward   H_l = ELU(H_{l-1} W_l^T + b_l)    one rslrl_linear_fwd launch per hidden layer; the last one
              Y   = H_{L-1} W_L^T + b_L         also computes the (<= 32 wide) output layer from its
                                                register tile (rslrl_linear_fwd_out)
    backward  dW_l = dZ_l^T H_{l-1}             x6 split-K weight-gradient kernel (rslrl_linear_wgrad)
              dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}) and db_{l-1} = column sums of dZ_{l-1}
                                                one rslrl_linear_dgrad_elu launch (+ a tiny fold); for the
                                                output layer together with its dW (rslrl_linear_dgrad_elu_wgrad)

so the pre-activations and dH never reach HBM and the separate ELU / ELU-backward / bias-reduction
kernels disappear.  Parameters, state_dict and the forward values are those of the nn.Sequential (the
MFMA accumulation order differs from hipBLASLt's at fp32 epsilon; tests/test_gpu_fused_mlp.py).
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..kernels import timer
from .linear import _splitk_weight_grad

MAX_WIDTH = 256


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


_FUSE_OUT = os.environ.get("RSLRL_FUSE_OUT", "1") == "1"  # output-layer backward in one launch
_FUSE_OUT_FWD = os.environ.get("RSLRL_FUSE_OUT_FWD", "1") == "1"  # output-layer forward in the last hidden GEMM
GEMM_F32 = 0  # v_mfma_f32_32x32x2_f32: exact f32 fma chain
GEMM_X6 = 1   # fp32 split into 3 bf16 planes, 6 bf16 MFMA products, fp32 accumulation (default)
_mode = GEMM_F32 if os.environ.get("RSLRL_GEMM_MODE", "x6") == "f32" else GEMM_X6


def set_gemm_mode(mode: int) -> int:
    """Select the arithmetic of the fused GEMMs (GEMM_F32 | GEMM_X6); returns the previous mode.  The
    initial mode comes from RSLRL_GEMM_MODE=f32|x6 (default x6)."""
    global _mode
    if mode not in (GEMM_F32, GEMM_X6):
        raise ValueError(f"unknown GEMM mode {mode}")
    prev, _mode = _mode, mode
    return prev


# B-operand images (include/rslrl_amd.h rslrl_linear_prepare_bimages).  Weights can change in place without
# moving their version counter (fused Adam does not bump it), so images are rebuilt on every use except
# inside a frozen_weights() scope, where the caller promises the weights do not change (the rollout).
_frozen_depth = 0
_bimage_cache: dict = {}


@contextlib.contextmanager
def frozen_weights():
    """Scope in which B images of weights are built once and reused (the rollout of on_policy_runner)."""
    global _frozen_depth
    _frozen_depth += 1
    try:
        yield
    finally:
        _frozen_depth -= 1
        if _frozen_depth == 0:
            _bimage_cache.clear()


def bimages(specs):
    """Images for [(w, transposed[, layout]), ...]: transposed=False -> B = w ([N, K]), True -> B = w^T;
    layout _lib.BIMAGE_LAYOUT_OUT -> the output-layer image of linear_fwd_out.  One launch for every image not
    already cached in a frozen_weights() scope."""
    out = [None] * len(specs)
    todo = []
    for i, spec in enumerate(specs):
        w, tr = spec[0], spec[1]
        layout = spec[2] if len(spec) > 2 else _lib.BIMAGE_LAYOUT_GEMM
        rows, depth = (w.shape[1], w.shape[0]) if tr else (w.shape[0], w.shape[1])
        key = (w.data_ptr(), tr, rows, depth, layout)
        if _frozen_depth:
            hit = _bimage_cache.get(key)
            if hit is not None and hit[0]() is w:
                out[i] = hit[1]
                continue
        todo.append((i, w, tr, rows, depth, key))
    if not todo:
        return out
    L = _lib.lib()
    sizes = [(L.rslrl_linear_out_image_bytes() if key[4] == _lib.BIMAGE_LAYOUT_OUT else
              L.rslrl_linear_bimage_bytes(depth)) // 4 for (_, _, _, _, depth, key) in todo]
    buf = torch.empty(sum(sizes), dtype=torch.float32, device=todo[0][1].device)
    for start in range(0, len(todo), _lib.MAX_BIMAGES):
        part = todo[start:start + _lib.MAX_BIMAGES]
        descs = (_lib.BImageDesc * len(part))()
        off = sum(sizes[:start])
        keep = []
        for d, (i, w, tr, rows, depth, key), n in zip(descs, part, sizes[start:start + len(part)]):
            src = w.detach()
            src = src if src.is_contiguous() else src.contiguous()
            keep.append(src)
            img = buf[off:off + n]
            off += n
            d.src, d.image, d.rows, d.depth, d.transposed = src.data_ptr(), img.data_ptr(), rows, depth, int(tr)
            d.layout = key[4]
            out[i] = img
            if _frozen_depth:
                _bimage_cache[key] = (weakref.ref(w), img)
        rc = L.rslrl_linear_prepare_bimages(descs, len(part), _stream(buf))
        _lib.check(rc, "rslrl_linear_prepare_bimages")
    return out


def bimage(w, transposed: bool):
    return bimages([(w, transposed)])[0]


def linear_fwd(x, w, b, elu: bool, img=None):
    """act(x w^T + b); img: B image of w (x6 arithmetic) or None (exact f32 MFMA)."""
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    with timer.span(f"linear_fwd[M={M},K={K},N={N}]", x.device, 4 * M * (K + N), 2 * M * K * N):
        rc = _lib.lib().rslrl_linear_fwd(x.data_ptr(), M, K, w.data_ptr(), N, b.data_ptr(), 1 if elu else 0,
                                         y.data_ptr(), img.data_ptr() if img is not None else None, _stream(x))
    _lib.check(rc, "rslrl_linear_fwd")
    return y


MAX_OUT_WIDTH = 32


def linear_fwd_out(x, w, b, img, w_out, b_out, out_img, store_h: bool):
    """(h, y): h = ELU(x w^T + b) (None unless store_h) and y = h w_out^T + b_out in one x6 launch; img: B image
    of w, out_img: the BIMAGE_LAYOUT_OUT image of w_out (<= 32 rows)."""
    M, K = x.shape
    N = w.shape[0]
    nout = w_out.shape[0]
    h = torch.empty(M, N, device=x.device, dtype=torch.float32) if store_h else None
    y = torch.empty(M, nout, device=x.device, dtype=torch.float32)
    flops = 2 * M * N * (K + nout)
    with timer.span(f"linear_fwd_out[M={M},K={K},N={N},out={nout}]", x.device,
                    4 * M * (K + nout + (N if store_h else 0)), flops):
        rc = _lib.lib().rslrl_linear_fwd_out(x.data_ptr(), M, K, b.data_ptr(), N, img.data_ptr(),
                                             h.data_ptr() if store_h else None, b_out.data_ptr(), nout,
                                             out_img.data_ptr(), y.data_ptr(), _stream(x))
    _lib.check(rc, "rslrl_linear_fwd_out")
    return h, y


def _fuse_out_fwd(ws) -> bool:
    """The last hidden layer and the output layer run as one linear_fwd_out launch (x6 only)."""
    return _FUSE_OUT_FWD and _mode == GEMM_X6 and len(ws) >= 2 and ws[-1].shape[0] <= MAX_OUT_WIDTH \
        and ws[-1].shape[1] % 4 == 0


def linear_dgrad_elu(dz, w, h, img=None):
    """(dz @ w) * ELU'(h) and its column sums; w is the layer weight [N, K] (dz [M, N], h [M, K]); img: B image
    of w^T (x6 arithmetic) or None (exact f32 MFMA)."""
    M, N = dz.shape
    K = w.shape[1]
    wt = w.t().contiguous() if img is None else w  # [K, N]: the f32 kernel's B operand rows are the output columns
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32)
    with timer.span(f"linear_dgrad[M={M},Nred={N},K={K}]", dz.device, 4 * M * (N + 2 * K), 2 * M * K * N):
        rc = L.rslrl_linear_dgrad_elu(dz.data_ptr(), M, N, wt.data_ptr(), K, h.data_ptr(), out.data_ptr(),
                                      part.data_ptr(), img.data_ptr() if img is not None else None, _stream(dz))
    _lib.check(rc, "rslrl_linear_dgrad_elu")
    db = torch.empty(K, device=dz.device, dtype=torch.float32)
    rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_column_sum_fold")
    return out, db


def linear_dgrad_elu_wgrad(dz, w, h, img):
    """Output-layer backward in one launch (x6; dz [M, Nred <= 16, % 4]): ((dz @ w) * ELU'(h), its column sums,
    dz^T h).  w is the layer weight [Nred, K] (only its image is read)."""
    M, N = dz.shape
    K = h.shape[1]
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32)
    wpart = torch.empty(tiles, N, K, device=dz.device, dtype=torch.float32)
    with timer.span(f"linear_dgrad_wgrad[M={M},Nred={N},K={K}]", dz.device, 4 * M * (N + 2 * K), 4 * M * K * N):
        rc = L.rslrl_linear_dgrad_elu_wgrad(dz.data_ptr(), M, N, K, h.data_ptr(), out.data_ptr(), part.data_ptr(),
                                            img.data_ptr(), wpart.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_linear_dgrad_elu_wgrad")
    db = torch.empty(K, device=dz.device, dtype=torch.float32)
    rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_column_sum_fold")
    dw = torch.empty(N, K, device=dz.device, dtype=torch.float32)
    nbytes = L.rslrl_fold_partials_workspace_bytes(tiles, N * K)
    ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=dz.device)
    rc = L.rslrl_fold_partials(wpart.data_ptr(), tiles, N * K, dw.data_ptr(), ws.data_ptr(), nbytes, _stream(dz))
    _lib.check(rc, "rslrl_fold_partials")
    return out, db, dw


def linear_wgrad(dz, x):
    """dz^T x ([N, K]) on the x6 weight-gradient kernel; dz [M, N], x [M, K], N, K <= 256 and 4-aligned."""
    M, N = dz.shape
    K = x.shape[1]
    L = _lib.lib()
    nbytes = L.rslrl_linear_wgrad_workspace_bytes(M, N, K)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dz.device)
    dw = torch.empty(N, K, dtype=torch.float32, device=dz.device)
    with timer.span(f"linear_wgrad[M={M},N={N},K={K}]", dz.device, 4 * M * (N + K), 2 * M * K * N):
        rc = L.rslrl_linear_wgrad(dz.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), ws.data_ptr(), nbytes,
                                  _stream(dz))
    _lib.check(rc, "rslrl_linear_wgrad")
    return dw


def _weight_grad(dz, x, x6: bool):
    # the x6 weight-gradient kernel computes TN x 256 tiles (TN = 32, 64 or 256 rows of its first operand):
    # the square hidden layers run it as dz^T x; the first layer (input width <= 64) as (x^T dz)^T on the
    # 64-row tiles; the narrow output layers stay on the split-K batched GEMM (networks/linear.py) unless
    # their backward is fused (linear_dgrad_elu_wgrad)
    if x6 and dz.shape[1] > 64 and x.shape[1] <= 64 and dz.shape[1] <= MAX_WIDTH and dz.shape[1] % 4 == 0:
        pad = (-x.shape[1]) % 4
        xp = F.pad(x, (0, pad)) if pad else x
        return linear_wgrad(xp, dz)[: x.shape[1]].t().contiguous()
    if x6 and dz.shape[1] > 32 and x.shape[1] > 64 and dz.shape[1] <= MAX_WIDTH and x.shape[1] <= MAX_WIDTH \
            and x.shape[1] % 4 == 0:
        pad = (-dz.shape[1]) % 4
        if pad:  # the critic's 1-wide output
            return linear_wgrad(F.pad(dz, (0, pad)), x)[: dz.shape[1]]
        return linear_wgrad(dz, x)
    return _splitk_weight_grad(dz, x)


class FusedMLPFunction(torch.autograd.Function):
    """y = MLP(x) for hidden ELU(alpha=1) layers; args: (x, W1, b1, ..., WL, bL)."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        hs = [x]
        h = x
        x6 = _mode == GEMM_X6
        nh = len(ws) - 1
        fuse_out = _fuse_out_fwd(ws)
        # forward images of the hidden layers + (for backward) the transposed images of layers 1..L-1
        # [+ the output-layer image]
        specs = [(w, False) for w in ws[:-1]] + [(w, True) for w in ws[1:]]
        if fuse_out:
            specs.append((ws[-1], False, _lib.BIMAGE_LAYOUT_OUT))
        imgs = bimages(specs) if x6 else [None] * (2 * nh)
        for l, (w, b, img) in enumerate(zip(ws[:-1], bs[:-1], imgs[:nh])):
            if fuse_out and l == nh - 1:
                h, y = linear_fwd_out(h, w, b, img, ws[-1], bs[-1], imgs[2 * nh], store_h=True)
            else:
                h = linear_fwd(h, w, b, elu=True, img=img)
            hs.append(h)
        ctx.dgrad_imgs = [None] + imgs[nh:2 * nh]  # index l: image of W_l^T
        ctx.x6 = x6
        if not fuse_out:
            y = F.linear(h, ws[-1], bs[-1])
        ctx.save_for_backward(*hs, *params)
        ctx.n_layers = len(ws)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = ctx.n_layers
        saved = ctx.saved_tensors
        hs, params = saved[:L], saved[L:]
        ws = params[0::2]
        grads_w = [None] * L
        grads_b = [None] * L
        dz = dy.contiguous()
        grads_b[L - 1] = dz.sum(0)
        for l in range(L - 1, -1, -1):
            h_in = hs[l]
            fuse_w = (_FUSE_OUT and ctx.x6 and l == L - 1 and l > 0 and dz.shape[1] <= 16 and h_in.shape[1] <= MAX_WIDTH
                      and ctx.needs_input_grad[1 + 2 * l])
            if fuse_w:  # output layer: dgrad + ELU' + bias grad + weight grad over one read of h (one launch)
                nred = dz.shape[1]
                pad = (-nred) % 4
                dzp = F.pad(dz, (0, pad)) if pad else dz
                dz, grads_b[l - 1], dw = linear_dgrad_elu_wgrad(dzp, ws[l], h_in, ctx.dgrad_imgs[l])
                grads_w[l] = dw[:nred]
                continue
            grads_w[l] = _weight_grad(dz, h_in, ctx.x6) if ctx.needs_input_grad[1 + 2 * l] else None
            if l == 0:
                dx = dz.mm(ws[0]) if ctx.needs_input_grad[0] else None
                break
            # dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}), db_{l-1} = column sums; a reduction width that is not a
            # multiple of 4 (the critic's 1-wide output) is zero-padded to the next multiple (the x6 image
            # zero-fills the weight side itself)
            w = ws[l]
            img = ctx.dgrad_imgs[l]
            pad = (-dz.shape[1]) % 4
            if pad:
                dz = F.pad(dz, (0, pad))
                if img is None:
                    w = F.pad(w, (0, 0, 0, pad))
            dz, grads_b[l - 1] = linear_dgrad_elu(dz, w, h_in, img)
        out = [dx]
        for gw, gb in zip(grads_w, grads_b):
            out += [gw, gb]
        return tuple(out)


def fusable_structure(mlp: nn.Sequential) -> bool:
    """Linear, ELU(alpha=1), ..., Linear[, Unflatten] with hidden widths <= 256, all widths 4-aligned."""
    mods = [m for m in mlp if not isinstance(m, nn.Unflatten)]
    if len(mods) < 3 or len(mods) % 2 == 0:
        return False
    for i, m in enumerate(mods):
        if i % 2 == 0:
            if not isinstance(m, nn.Linear) or m.bias is None:
                return False
        elif not (isinstance(m, nn.ELU) and m.alpha == 1.0 and not m.inplace):
            return False
    linears = mods[0::2]
    if linears[0].in_features % 4:
        return False
    return all(m.out_features <= MAX_WIDTH and m.out_features % 4 == 0 for m in linears[:-1])


def fusable(mlp: nn.Sequential, x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and fusable_structure(mlp)


def fused_mlp_forward(mlp: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    linears = [m for m in mlp if isinstance(m, nn.Linear)]
    params = []
    for m in linears:
        params += [m.weight, m.bias]
    x = x if x.is_contiguous() else x.contiguous()
    if torch.is_grad_enabled() and any(p.requires_grad for p in params + [x]):
        y = FusedMLPFunction.apply(x, *params)
    else:
        h = x
        nh = len(linears) - 1
        ws = [m.weight for m in linears]
        fuse_out = _fuse_out_fwd(ws)
        specs = [(w, False) for w in ws[:-1]]
        if fuse_out:
            specs.append((ws[-1], False, _lib.BIMAGE_LAYOUT_OUT))
        imgs = bimages(specs) if _mode == GEMM_X6 else [None] * nh
        y = None
        for l, (m, img) in enumerate(zip(linears[:-1], imgs)):
            if fuse_out and l == nh - 1:  # the last activation never reaches HBM
                _, y = linear_fwd_out(h, m.weight, m.bias, img, ws[-1], linears[-1].bias, imgs[nh], store_h=False)
            else:
                h = linear_fwd(h, m.weight, m.bias, elu=True, img=img)
        if y is None:
            y = F.linear(h, linears[-1].weight, linears[-1].bias)
    for m in mlp:
        if isinstance(m, nn.Unflatten):
            y = m(y)
    return y
