"""MLP network (rsl_rl/networks/mlp.py:15-120).

An nn.Sequential of Linear + activation blocks whose module indices ("0", "2", ...) match the
reference, so state_dict keys (actor.0.weight, ...) and checkpoints are interchangeable.  On a ROCm
device a Linear+ELU stack runs on the fused fp32 MFMA kernels of networks/fused_mlp.py (bias+ELU in the
GEMM epilogue, ELU'+bias-gradient in the data-gradient epilogue, split-K weight gradients); any other
structure runs layer by layer through PyTorch-ROCm with the split-K weight gradient (networks/linear.py).
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..utils import resolve_nn_activation
from .fused_mlp import fusable_structure, fused_mlp_forward
from .linear import linear


class MLP(nn.Sequential):
    """Linear/activation stack.  A hidden dim of -1 means "same as the input dim"; a tuple/list output
    dim adds an Unflatten to that shape (e.g. [2, A] for state-dependent std)."""

    def __init__(self, input_dim: int, output_dim, hidden_dims, activation: str = "elu",
                 last_activation: str | None = None):
        super().__init__()
        dims = [input_dim] + [input_dim if d == -1 else d for d in hidden_dims]
        act = resolve_nn_activation(activation)
        layers: list[nn.Module] = []
        for d_in, d_out in zip(dims[:-1], dims[1:]):
            layers += [nn.Linear(d_in, d_out), act]
        if isinstance(output_dim, int):
            layers.append(nn.Linear(dims[-1], output_dim))
        else:
            layers.append(nn.Linear(dims[-1], math.prod(output_dim)))
            layers.append(nn.Unflatten(dim=-1, unflattened_size=tuple(output_dim)))
        if last_activation is not None:
            layers.append(resolve_nn_activation(last_activation))
        for i, layer in enumerate(layers):
            self.add_module(str(i), layer)
        self._fused = fusable_structure(self)

    def init_weights(self, scales):
        """Orthogonal weights with per-layer gain (scales indexed by module index) and zero biases."""
        for idx, module in enumerate(self):
            if isinstance(module, nn.Linear):
                gain = scales[idx] if isinstance(scales, (list, tuple)) else scales
                nn.init.orthogonal_(module.weight, gain=gain)
                nn.init.zeros_(module.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # Linear+ELU stacks on a ROCm device run on the fused MFMA kernels (networks/fused_mlp.py)
        if self._fused and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32:
            return fused_mlp_forward(self, x)
        for layer in self:
            x = linear(x, layer.weight, layer.bias) if isinstance(layer, nn.Linear) else layer(x)
        return x

    def reset(self, dones=None, hidden_states=None):
        pass

    def detach_hidden_states(self, dones=None):
        pass
