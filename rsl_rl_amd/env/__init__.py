"""Environment interface (mirrors rsl_rl.env) + the synthetic benchmark environment."""

from .synthetic import SyntheticVecEnv
from .vec_env import VecEnv

__all__ = ["VecEnv", "SyntheticVecEnv"]
