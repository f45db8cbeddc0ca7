"""Network building blocks (mirrors rsl_rl.networks for the PPO path)."""

from .mlp import MLP
from .normalization import EmpiricalDiscountedVariationNormalization, EmpiricalNormalization

__all__ = ["MLP", "EmpiricalNormalization", "EmpiricalDiscountedVariationNormalization"]
