"""Learning algorithms (mirrors rsl_rl.algorithms for PPO)."""

from .ppo import PPO

__all__ = ["PPO"]
