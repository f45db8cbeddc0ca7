"""Policy modules (mirrors rsl_rl.modules for the PPO path)."""

from .actor_critic import ActorCritic
from .rnd import RandomNetworkDistillation, resolve_rnd_config
from .symmetry import resolve_symmetry_config

__all__ = ["ActorCritic", "RandomNetworkDistillation", "resolve_rnd_config", "resolve_symmetry_config"]
