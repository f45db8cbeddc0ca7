"""Rollout storage (mirrors rsl_rl.storage)."""

from .rollout_storage import RolloutStorage

__all__ = ["RolloutStorage"]
