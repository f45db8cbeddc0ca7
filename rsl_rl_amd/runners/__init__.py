"""Runners (mirrors rsl_rl.runners for PPO)."""

from .on_policy_runner import OnPolicyRunner

__all__ = ["OnPolicyRunner"]
