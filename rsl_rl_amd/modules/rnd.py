"""Random Network Distillation intrinsic reward (rsl_rl/modules/rnd.py:14-209).

Same module layout (predictor / target MLPs, optional state and reward normalisers, weight schedules)
and state_dict keys as the reference.  During the rollout the predictor/target forward, the
intrinsic reward and its add to the extrinsic reward run inside the fused record kernel
(csrc/rollout.hip via PPO.process_env_step) whenever the networks have the one-hidden-layer ELU form
and reward normalisation is off; the PyTorch forward here serves every other case and the update's
predictor loss.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from ..networks import MLP, EmpiricalDiscountedVariationNormalization, EmpiricalNormalization


class RandomNetworkDistillation(nn.Module):
    """Intrinsic reward = weight * || target(s) - predictor(s) ||_2 (Burda et al., 2018)."""

    def __init__(
        self,
        num_states: int,
        obs_groups: dict,
        num_outputs: int,
        predictor_hidden_dims: list,
        target_hidden_dims: list,
        activation: str = "elu",
        weight: float = 0.0,
        state_normalization: bool = False,
        reward_normalization: bool = False,
        device: str = "cpu",
        weight_schedule: dict | None = None,
    ):
        super().__init__()
        self.num_states = num_states
        self.obs_groups = obs_groups
        self.num_outputs = num_outputs
        self.initial_weight = weight
        self.weight = weight
        self.device = device
        self.state_normalization = state_normalization
        self.reward_normalization = reward_normalization
        self.state_normalizer = (
            EmpiricalNormalization(shape=[num_states], until=1.0e8).to(device) if state_normalization else nn.Identity()
        )
        self.reward_normalizer = (
            EmpiricalDiscountedVariationNormalization(shape=[], until=1.0e8).to(device)
            if reward_normalization
            else nn.Identity()
        )
        self.update_counter = 0
        if weight_schedule is not None:
            self.weight_scheduler_params = weight_schedule
            self.weight_scheduler = getattr(self, f"_{weight_schedule['mode']}_weight_schedule")
        else:
            self.weight_scheduler = None
        self.predictor = MLP(num_states, num_outputs, predictor_hidden_dims, activation).to(device)
        self.target = MLP(num_states, num_outputs, target_hidden_dims, activation).to(device)
        self.target.eval()

    def get_intrinsic_reward(self, obs) -> torch.Tensor:
        self.update_counter += 1  # counts env steps per learning iteration
        state = self.state_normalizer(self.get_rnd_state(obs))
        target = self.target(state).detach()
        pred = self.predictor(state).detach()
        reward = self.reward_normalizer(torch.linalg.norm(target - pred, dim=1))
        if self.weight_scheduler is not None:
            self.weight = self.weight_scheduler(step=self.update_counter, **self.weight_scheduler_params)
        else:
            self.weight = self.initial_weight
        reward *= self.weight
        return reward

    def forward(self, *args, **kwargs):
        raise RuntimeError("Forward method is not implemented. Use get_intrinsic_reward instead.")

    def train(self, mode: bool = True):
        self.predictor.train(mode)
        if self.state_normalization:
            self.state_normalizer.train(mode)
        if self.reward_normalization:
            self.reward_normalizer.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def get_rnd_state(self, obs):
        return torch.cat([obs[g] for g in self.obs_groups["rnd_state"]], dim=-1)

    def update_normalization(self, obs):
        if self.state_normalization:
            self.state_normalizer.update(self.get_rnd_state(obs))

    # weight schedules (rnd.py:168-182)
    def _constant_weight_schedule(self, step: int, **kwargs):
        return self.initial_weight

    def _step_weight_schedule(self, step: int, final_step: int, final_value: float, **kwargs):
        return self.initial_weight if step < final_step else final_value

    def _linear_weight_schedule(self, step: int, initial_step: int, final_step: int, final_value: float, **kwargs):
        if step < initial_step:
            return self.initial_weight
        if step > final_step:
            return final_value
        # left to right as the reference evaluates it: ((final - init) * (step - i0)) / (f - i0), then + init
        span = final_value - self.initial_weight
        return self.initial_weight + span * (step - initial_step) / (final_step - initial_step)


def resolve_rnd_config(alg_cfg, obs, obs_groups, env):
    """Fill num_states / obs_groups of rnd_cfg and scale its weight by env.unwrapped.step_dt (rnd.py:185-209)."""
    if alg_cfg.get("rnd_cfg") is not None:
        num = 0
        for g in obs_groups["rnd_state"]:
            assert len(obs[g].shape) == 2, "The RND module only supports 1D observations."
            num += obs[g].shape[-1]
        alg_cfg["rnd_cfg"]["num_states"] = num
        alg_cfg["rnd_cfg"]["obs_groups"] = obs_groups
        alg_cfg["rnd_cfg"]["weight"] *= env.unwrapped.step_dt
    return alg_cfg
