"""Helper functions (mirrors rsl_rl.utils for the PPO path)."""

from .tensordict import TensorDict
from .utils import (
    resolve_nn_activation,
    resolve_obs_groups,
    resolve_optimizer,
    store_code_state,
    string_to_callable,
)

__all__ = [
    "TensorDict",
    "resolve_nn_activation",
    "resolve_obs_groups",
    "resolve_optimizer",
    "store_code_state",
    "string_to_callable",
]
