"""Synthetic VecEnv for benchmarks and tests.

Observations ~ N(0, 1) [N, O] per group, rewards ~ N(0, 1) [N], dones ~ Bernoulli(done_prob) as
int64 [N], extras["time_outs"] ~ Bernoulli(timeout_prob) restricted to done envs.  All draws come from
a per-instance generator on the env's device seeded with `seed`, so the stream does not touch the
global RNG state.  `unwrapped.step_dt` is provided for the RND weight scaling (rnd.py:208).
"""

from __future__ import annotations

import os

import torch

from ..utils import TensorDict
from .vec_env import VecEnv


class SyntheticVecEnv(VecEnv):
    kRing = 3  # fused step: output buffer sets reused round-robin

    def __init__(self, num_envs: int, num_obs: int, num_actions: int, device="cpu", *, seed: int = 0,
                 num_privileged_obs: int = 0, done_prob: float = 0.02, timeout_prob: float = 0.0,
                 max_episode_length: int = 1000, step_dt: float = 0.02):
        self.num_envs = num_envs
        self.num_obs = num_obs
        self.num_privileged_obs = num_privileged_obs
        self.num_actions = num_actions
        self.device = torch.device(device)
        self.max_episode_length = max_episode_length
        self.episode_length_buf = torch.zeros(num_envs, dtype=torch.long, device=self.device)
        self.done_prob = done_prob
        self.timeout_prob = timeout_prob
        self.step_dt = step_dt
        self.cfg = {"num_envs": num_envs, "num_obs": num_obs, "num_actions": num_actions}
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self._obs = self._draw_obs()
        # on a ROCm device one step is one launch (rslrl_synthetic_env_step: the same distributions and done /
        # time-out / episode-length rules from a counter-based generator keyed by `seed`); CPU tensors and
        # privileged observation groups keep the torch implementation below
        self._fused = (self.device.type == "cuda" and num_privileged_obs == 0 and num_obs % 4 == 0
                       and os.environ.get("RSLRL_SYNTH_ENV", "fused") != "torch")
        self._seed = int(seed)
        self._step_count = 0
        self._ring = None  # the fused step's output buffer sets (allocated at the first step)

    @property
    def unwrapped(self):
        return self

    def _draw_obs(self):
        groups = {"policy": torch.randn(self.num_envs, self.num_obs, generator=self.gen, device=self.device)}
        if self.num_privileged_obs:
            groups["privileged"] = torch.randn(self.num_envs, self.num_privileged_obs, generator=self.gen,
                                               device=self.device)
        return TensorDict(groups, batch_size=[self.num_envs], device=self.device)

    def get_observations(self):
        return self._obs

    def step(self, actions: torch.Tensor):
        if self._fused:
            return self._step_fused()
        n = self.num_envs
        self._obs = self._draw_obs()
        rewards = torch.randn(n, generator=self.gen, device=self.device)
        u = torch.rand(n, generator=self.gen, device=self.device)
        dones = (u < self.done_prob).to(torch.long)
        self.episode_length_buf += 1
        if self.timeout_prob > 0:
            time_outs = (u < self.done_prob * self.timeout_prob).to(torch.float32)
        else:
            time_outs = torch.zeros(n, device=self.device)
        over = self.episode_length_buf >= self.max_episode_length
        dones = torch.where(over, torch.ones_like(dones), dones)
        time_outs = torch.where(over, torch.ones_like(time_outs), time_outs)
        self.episode_length_buf = torch.where(dones > 0, torch.zeros_like(self.episode_length_buf),
                                              self.episode_length_buf)
        return self._obs, rewards, dones, {"time_outs": time_outs}

    def _step_fused(self):
        from ..kernels import _stream

        n, dev = self.num_envs, self.device
        # outputs from a ring of kRing buffer sets: a step's tensors stay valid for the next kRing - 1 steps (the runner
        # consumes them within one; a ring instead of four allocations and a TensorDict per step: ~10 us of host time
        # on the launch-bound rollout of a small per-GPU share)
        if self._ring is None:
            from .. import _lib

            self._step_fn = _lib.lib().rslrl_synthetic_env_step
            self._check = _lib.check
            self._ring = []
            for _ in range(self.kRing):
                obs = torch.empty(n, self.num_obs, device=dev)
                bufs = (TensorDict({"policy": obs}, batch_size=[n], device=dev), obs, torch.empty(n, device=dev),
                        torch.empty(n, dtype=torch.long, device=dev), torch.empty(n, device=dev))
                ptrs = (bufs[1].data_ptr(), bufs[2].data_ptr(), bufs[3].data_ptr(), bufs[4].data_ptr())
                self._ring.append((bufs, ptrs, {"time_outs": bufs[4]}))
        self._step_count += 1
        bufs, ptrs, extras = self._ring[self._step_count % self.kRing]
        rc = self._step_fn(
            ptrs[0], self.num_obs, ptrs[1], ptrs[2], ptrs[3], self.episode_length_buf.data_ptr(), n, self._seed,
            self._step_count & 0xFFFFFFFF, float(self.done_prob), float(self.timeout_prob), int(self.max_episode_length),
            _stream(dev))
        self._check(rc, "rslrl_synthetic_env_step")
        self._obs = bufs[0]
        return self._obs, bufs[2], bufs[3], dict(extras)
