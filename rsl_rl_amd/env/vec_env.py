"""Vectorised-environment interface (rsl_rl/env/vec_env.py:13-108), unchanged so Isaac Lab /
Legged-Gym environments plug in as they are."""

from __future__ import annotations

from abc import ABC, abstractmethod

import torch


class VecEnv(ABC):
    """A batch of synchronised environments.

    Attributes: num_envs, num_actions, max_episode_length (int or per-env tensor), episode_length_buf,
    device, cfg.  step() returns (observations TensorDict, rewards [N], dones [N], extras) where extras
    may hold "time_outs" [N] (truncations, bootstrapped in PPO.process_env_step) and "episode"/"log".
    Observation groups are mapped to the policy / critic / rnd_state sets by the runner's obs_groups.
    """

    num_envs: int
    num_actions: int
    max_episode_length: int | torch.Tensor
    episode_length_buf: torch.Tensor
    device: torch.device | str
    cfg: dict | object

    @abstractmethod
    def get_observations(self):
        """Current observations as a TensorDict of observation groups."""
        raise NotImplementedError

    @abstractmethod
    def step(self, actions: torch.Tensor):
        """Apply actions [num_envs, num_actions]; return (obs, rewards, dones, extras)."""
        raise NotImplementedError
