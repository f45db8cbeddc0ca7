"""Actor/critic MLP forward + backward on the fused fp32 MFMA GEMMs.

For an `MLP` of Linear(+ELU) hidden blocks and a final Linear (rsl_rl/networks/mlp.py:59-114) this
autograd Function runs

    forward   H_l = ELU(H_{l-1} W_l^T + b_l)    one rslrl_linear_fwd launch per hidden layer
              Y   = H_{L-1} W_L^T + b_L         F.linear (the 1-12 wide output layer suits hipBLASLt)
    backward  dW_l = dZ_l^T H_{l-1}             split-K batched GEMM (networks/linear.py)
              dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}) and db_{l-1} = column sums of dZ_{l-1}
                                                one rslrl_linear_dgrad_elu launch (+ a tiny fold)

so the pre-activations and dH never reach HBM and the separate ELU / ELU-backward / bias-reduction
kernels disappear.  Parameters, state_dict and the forward values are those of the nn.Sequential (the
fp32 MFMA accumulation order differs from hipBLASLt's at fp32 epsilon; tests/test_gpu_fused_mlp.py).
"""

from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from .linear import _splitk_weight_grad

MAX_WIDTH = 256


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def linear_fwd(x, w, b, elu: bool):
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    rc = _lib.lib().rslrl_linear_fwd(x.data_ptr(), M, K, w.data_ptr(), N, b.data_ptr(), 1 if elu else 0,
                                     y.data_ptr(), _stream(x))
    _lib.check(rc, "rslrl_linear_fwd")
    return y


def linear_dgrad_elu(dz, w, h):
    """(dz @ w) * ELU'(h) and its column sums; w is the layer weight [N, K] (dz [M, N], h [M, K])."""
    M, N = dz.shape
    K = w.shape[1]
    wt = w.t().contiguous()  # [K, N]: the kernel's B operand rows are the output columns
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32)
    rc = L.rslrl_linear_dgrad_elu(dz.data_ptr(), M, N, wt.data_ptr(), K, h.data_ptr(), out.data_ptr(),
                                  part.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_linear_dgrad_elu")
    db = torch.empty(K, device=dz.device, dtype=torch.float32)
    rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_column_sum_fold")
    return out, db


class FusedMLPFunction(torch.autograd.Function):
    """y = MLP(x) for hidden ELU(alpha=1) layers; args: (x, W1, b1, ..., WL, bL)."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        hs = [x]
        h = x
        for w, b in zip(ws[:-1], bs[:-1]):
            h = linear_fwd(h, w, b, elu=True)
            hs.append(h)
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
            grads_w[l] = _splitk_weight_grad(dz, h_in) if ctx.needs_input_grad[1 + 2 * l] else None
            if l == 0:
                dx = dz.mm(ws[0]) if ctx.needs_input_grad[0] else None
                break
            # dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}), db_{l-1} = column sums; a reduction width that is not a
            # multiple of 4 (the critic's 1-wide output) is zero-padded to the next multiple
            w = ws[l]
            pad = (-dz.shape[1]) % 4
            if pad:
                dz = F.pad(dz, (0, pad))
                w = F.pad(w, (0, 0, 0, pad))
            dz, grads_b[l - 1] = linear_dgrad_elu(dz, w, h_in)
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
        for m in linears[:-1]:
            h = linear_fwd(h, m.weight, m.bias, elu=True)
        y = F.linear(h, linears[-1].weight, linears[-1].bias)
    for m in mlp:
        if isinstance(m, nn.Unflatten):
            y = m(y)
    return y
