"""Running observation / reward normalisers (rsl_rl/networks/normalization.py).

Same buffers (_mean, _var, _std, count) and update rule as the reference so checkpoints load into
either implementation.  On a ROCm device the update, the forward and the reward normaliser run on the
HIP kernels of csrc/normalizer.hip (fp64 batch moments, the reference's fp32
update order, the `until` limit tested on the device -- no host synchronisation); CPU modules (e.g. an
exported inference policy) keep the PyTorch expressions.
"""

from __future__ import annotations

import torch
from torch import nn

from .. import _lib


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class _WS:
    bufs: dict = {}

    @classmethod
    def get(cls, device, nbytes):
        b = cls.bufs.get(device)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
            cls.bufs[device] = b
        return b


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
        if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.stride(-1) == 1:
            N, D = x.shape
            y = torch.empty(N, D, dtype=torch.float32, device=x.device)
            rc = _lib.lib().rslrl_normalizer_apply(x.data_ptr(), N, D, x.stride(0), self._mean.data_ptr(),
                                                   self._std.data_ptr(), float(self.eps), y.data_ptr(), _stream(x))
            _lib.check(rc, "rslrl_normalizer_apply")
            return y
        return (x - self._mean) / (self._std + self.eps)

    @torch.jit.unused
    def update(self, x):
        """Chan et al. parallel-moments merge of the batch into the running (mean, var)."""
        if not self.training:
            return
        if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.stride(-1) == 1 and x.shape[1] <= 256:
            N, D = x.shape
            L = _lib.lib()
            nbytes = L.rslrl_normalizer_workspace_bytes(N, D)
            ws = _WS.get(x.device, nbytes)
            until = -1 if self.until is None else int(self.until)
            rc = L.rslrl_normalizer_update(x.data_ptr(), N, D, x.stride(0), self._mean.data_ptr(), self._var.data_ptr(),
                                           self._std.data_ptr(), self.count.data_ptr(), until, ws.data_ptr(), nbytes,
                                           _stream(x))
            _lib.check(rc, "rslrl_normalizer_update")
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
        en = self.emp_norm
        if rew.is_cuda and rew.dim() == 1 and rew.dtype == torch.float32 and rew.is_contiguous():
            N = rew.shape[0]
            first = self.disc_avg.avg is None
            if self.training and first:
                self.disc_avg.avg = torch.empty_like(rew)
            L = _lib.lib()
            nbytes = L.rslrl_normalizer_workspace_bytes(N, 1)
            ws = _WS.get(rew.device, nbytes)
            out = torch.empty_like(rew)
            until = -1 if en.until is None else int(en.until)
            avg = self.disc_avg.avg
            rc = L.rslrl_reward_normalize(rew.data_ptr(), N, float(self.disc_avg.gamma),
                                          avg.data_ptr() if avg is not None else None, int(first),
                                          en._mean.data_ptr(), en._var.data_ptr(), en._std.data_ptr(),
                                          en.count.data_ptr(), until, int(self.training), out.data_ptr(),
                                          ws.data_ptr(), nbytes, _stream(rew))
            _lib.check(rc, "rslrl_reward_normalize")
            return out
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
