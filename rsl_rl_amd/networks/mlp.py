"""MLP network (rsl_rl/networks/mlp.py:15-120).

An nn.Sequential of Linear + activation blocks whose module indices ("0", "2", ...) match the
reference, so state_dict keys (actor.0.weight, ...) and checkpoints are interchangeable.  The GEMMs run
through PyTorch-ROCm (hipBLASLt) with the weight gradient as a split-K batched GEMM (networks/linear.py);
fusing the whole MLP onto MFMA is a later step.
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..utils import resolve_nn_activation
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

    def init_weights(self, scales):
        """Orthogonal weights with per-layer gain (scales indexed by module index) and zero biases."""
        for idx, module in enumerate(self):
            if isinstance(module, nn.Linear):
                gain = scales[idx] if isinstance(scales, (list, tuple)) else scales
                nn.init.orthogonal_(module.weight, gain=gain)
                nn.init.zeros_(module.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for layer in self:
            x = linear(x, layer.weight, layer.bias) if isinstance(layer, nn.Linear) else layer(x)
        return x

    def reset(self, dones=None, hidden_states=None):
        pass

    def detach_hidden_states(self, dones=None):
        pass
