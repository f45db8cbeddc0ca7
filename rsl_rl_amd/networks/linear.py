"""Linear layer whose weight gradient is a split-K batched GEMM.

In PPO the MLP batch is a whole mini-batch (C3: 393,216 rows) while the layers are small (<= 256 x 256),
so the weight gradient dW = dY^T X is a GEMM with a tiny [out, in] output and a 393k-deep reduction.
hipBLASLt runs that shape on ~100 workgroups (the output tile count) and reaches 3-54 TFLOP/s on MI355X
(scripts/dw_gemm_probe.py: 256x256 at 54, 256x48 at 11, 12x256 at 3).  Splitting the rows into S
slices turns it into one batched GEMM with S x more workgroups plus an S-way sum of tiny partials:
256x256 reaches 141 TFLOP/s (fp32 MFMA peak 157) and the whole MLP backward ~2.5x faster.

The forward and dX are the plain GEMMs torch would run; only the reduction order of dW / db changes
(S fp32 partial sums instead of one running sum), well inside fp32 tolerance.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

ROWS_PER_SLICE = 3072  # ~128 slices at C3's 393,216-row mini-batch


def _splitk_weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dy^T x for dy [B, out], x [B, in] with a split-K batched GEMM (+ a plain GEMM for the tail)."""
    B = x.shape[0]
    slices = B // ROWS_PER_SLICE
    if slices < 2:
        return dy.t().mm(x)
    main = slices * ROWS_PER_SLICE
    xs = x[:main].view(slices, ROWS_PER_SLICE, x.shape[1])
    dys = dy[:main].view(slices, ROWS_PER_SLICE, dy.shape[1])
    dw = torch.bmm(dys.transpose(1, 2), xs).sum(0)
    if main < B:
        dw += dy[main:].t().mm(x[main:])
    return dw


class SplitKLinearFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy.mm(weight) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            dy2 = dy.reshape(-1, dy.shape[-1])
            dw = _splitk_weight_grad(dy2, x2 if x2.is_contiguous() else x2.contiguous())
        db = dy.reshape(-1, dy.shape[-1]).sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        if dx is not None:
            dx = dx.view(x.shape)
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """F.linear with the split-K weight gradient when autograd will need it on a ROCm device."""
    if x.is_cuda and torch.is_grad_enabled() and (weight.requires_grad or x.requires_grad) and x.dim() == 2:
        return SplitKLinearFunction.apply(x, weight, bias)
    return F.linear(x, weight, bias)
