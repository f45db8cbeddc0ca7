"""TensorDict type used for observations.

Isaac Lab / Legged-Gym hand the runner `tensordict.TensorDict` objects (vec_env.py:49-58); when the
`tensordict` package is installed it is used as is.  This image does not ship it, so a minimal keyed
container with the same subset of behaviour the PPO path relies on (string lookup, row indexing that
returns views, copy_, flatten, to, batch_size) stands in.
"""

from __future__ import annotations

import math

import torch

try:  # pragma: no cover - exercised only where tensordict is installed
    from tensordict import TensorDict  # type: ignore
except ImportError:  # pragma: no cover - the branch taken in this image

    class TensorDict:  # type: ignore[no-redef]
        """Dict of tensors sharing leading batch dimensions."""

        def __init__(self, source=None, batch_size=None, device=None):
            self._d = dict(source or {})
            if batch_size is None:
                first = next(iter(self._d.values()))
                batch_size = [first.shape[0]]
            self.batch_size = torch.Size(batch_size)
            self.device = torch.device(device) if device is not None else None

        # -- mapping interface
        def __getitem__(self, key):
            if isinstance(key, str):
                return self._d[key]
            out = {k: v[key] for k, v in self._d.items()}
            nb = len(self.batch_size) - (1 if isinstance(key, int) else 0)
            if out:
                first = next(iter(out.values()))
                bs = list(first.shape[: max(nb, 0)])
            else:
                bs = []
            return TensorDict(out, batch_size=bs, device=self.device)

        def __setitem__(self, key, value):
            if isinstance(key, str):
                self._d[key] = value
            else:
                for k, v in self._d.items():
                    v[key] = value[k]

        def __contains__(self, key):
            return key in self._d

        def __iter__(self):
            return iter(self._d)

        def __len__(self):
            return len(self._d)

        def keys(self):
            return self._d.keys()

        def values(self):
            return self._d.values()

        def items(self):
            return self._d.items()

        def get(self, key, default=None):
            return self._d.get(key, default)

        # -- tensor-like interface
        @property
        def shape(self):
            return self.batch_size

        def copy_(self, other):
            for k, v in self._d.items():
                v.copy_(other[k])
            return self

        def flatten(self, start_dim, end_dim):
            out = {k: v.flatten(start_dim, end_dim) for k, v in self._d.items()}
            bs = list(self.batch_size)
            bs = bs[:start_dim] + [math.prod(bs[start_dim:end_dim + 1])] + bs[end_dim + 1:]
            return TensorDict(out, batch_size=bs, device=self.device)

        def to(self, device, non_blocking=False):
            return TensorDict({k: v.to(device, non_blocking=non_blocking) for k, v in self._d.items()},
                              batch_size=self.batch_size, device=device)

        def clone(self):
            return TensorDict({k: v.clone() for k, v in self._d.items()}, batch_size=self.batch_size,
                              device=self.device)

        def detach(self):
            return TensorDict({k: v.detach() for k, v in self._d.items()}, batch_size=self.batch_size,
                              device=self.device)

        def __repr__(self):
            fields = ", ".join(f"{k}: {tuple(v.shape)}" for k, v in self._d.items())
            return f"TensorDict({fields}; batch_size={list(self.batch_size)})"

__all__ = ["TensorDict"]
