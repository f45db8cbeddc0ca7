"""Running observation / reward normalisers (rsl_rl/networks/normalization.py).

Same buffers (_mean, _var, _std, count) and update rule as the reference so checkpoints load into
either implementation.  Fusing the per-step moment update into the rollout-side kernel is listed as a
"next" item in SURVEY.md §8f.
"""

from __future__ import annotations

import torch
from torch import nn


class EmpiricalNormalization(nn.Module):
    """(x - mean) / (std + eps) with running moments over all samples seen (normalization.py:14-72)."""

    def __init__(self, shape, eps=1e-2, until=None):
        super().__init__()
        self.eps = eps
        self.until = until
        self.register_buffer("_mean", torch.zeros(shape).unsqueeze(0))
        self.register_buffer("_var", torch.ones(shape).unsqueeze(0))
        self.register_buffer("_std", torch.ones(shape).unsqueeze(0))
        self.register_buffer("count", torch.tensor(0, dtype=torch.long))

    @property
    def mean(self):
        return self._mean.squeeze(0).clone()

    @property
    def std(self):
        return self._std.squeeze(0).clone()

    def forward(self, x):
        return (x - self._mean) / (self._std + self.eps)

    @torch.jit.unused
    def update(self, x):
        """Chan et al. parallel-moments merge of the batch into the running (mean, var)."""
        if not self.training:
            return
        if self.until is not None and self.count >= self.until:
            return
        n = x.shape[0]
        self.count += n
        rate = n / self.count
        batch_var = torch.var(x, dim=0, unbiased=False, keepdim=True)
        batch_mean = torch.mean(x, dim=0, keepdim=True)
        delta = batch_mean - self._mean
        self._mean += rate * delta
        self._var += rate * (batch_var - self._var + delta * (batch_mean - self._mean))
        self._std = torch.sqrt(self._var)

    @torch.jit.unused
    def inverse(self, y):
        return y * (self._std + self.eps) + self._mean


class EmpiricalDiscountedVariationNormalization(nn.Module):
    """Divide rewards by the running std of their discounted sum (Pathak et al.; normalization.py:75-105)."""

    def __init__(self, shape, eps=1e-2, gamma=0.99, until=None):
        super().__init__()
        self.emp_norm = EmpiricalNormalization(shape, eps, until)
        self.disc_avg = _DiscountedAverage(gamma)

    def forward(self, rew):
        if self.training:
            self.emp_norm.update(self.disc_avg.update(rew))
        if self.emp_norm._std > 0:
            return rew / self.emp_norm._std
        return rew


class _DiscountedAverage:
    """R_t = gamma * R_{t-1} + r_t (normalization.py:108-130)."""

    def __init__(self, gamma):
        self.avg = None
        self.gamma = gamma

    def update(self, rew: torch.Tensor) -> torch.Tensor:
        self.avg = rew if self.avg is None else self.avg * self.gamma + rew
        return self.avg
