"""Configuration helpers with the reference's semantics (rsl_rl/utils/utils.py).

Only the helpers the PPO path needs are provided: activation / optimizer lookup, `module:attr`
resolution, observation-set resolution, and the git code-state snapshot used by the runner.
Trajectory padding for recurrent policies (utils.py:78-141) is outside this build's scope.
"""

from __future__ import annotations

import importlib
import os
import pathlib
import subprocess
import warnings
from typing import Callable

import torch

_ACTIVATIONS = {
    "elu": torch.nn.ELU,
    "selu": torch.nn.SELU,
    "relu": torch.nn.ReLU,
    "crelu": torch.nn.CELU,
    "lrelu": torch.nn.LeakyReLU,
    "tanh": torch.nn.Tanh,
    "sigmoid": torch.nn.Sigmoid,
    "softplus": torch.nn.Softplus,
    "gelu": torch.nn.GELU,
    "swish": torch.nn.SiLU,
    "mish": torch.nn.Mish,
    "identity": torch.nn.Identity,
}

_OPTIMIZERS = {
    "adam": torch.optim.Adam,
    "adamw": torch.optim.AdamW,
    "sgd": torch.optim.SGD,
    "rmsprop": torch.optim.RMSprop,
}


def resolve_nn_activation(act_name: str) -> torch.nn.Module:
    """Activation module by (case-insensitive) name; ValueError listing the valid names otherwise.

    Mirrors rsl_rl/utils/utils.py:18-49.
    """
    key = act_name.lower()
    if key not in _ACTIVATIONS:
        raise ValueError(f"Invalid activation function '{act_name}'. Valid activations are: {list(_ACTIVATIONS)}")
    return _ACTIVATIONS[key]()


def resolve_optimizer(optimizer_name: str):
    """Optimizer class by name (utils.py:52-75)."""
    key = optimizer_name.lower()
    if key not in _OPTIMIZERS:
        raise ValueError(f"Invalid optimizer '{optimizer_name}'. Valid optimizers are: {list(_OPTIMIZERS)}")
    return _OPTIMIZERS[key]


def string_to_callable(name: str) -> Callable:
    """Resolve 'package.module:attribute' to a callable (utils.py:172-199)."""
    try:
        mod_name, attr_name = name.split(":")
        obj = getattr(importlib.import_module(mod_name), attr_name)
    except AttributeError as e:
        raise ValueError(
            "We could not interpret the entry as a callable object. The format of input should be"
            f" 'module:attribute_name'\nWhile processing input '{name}', received the error:\n {e}."
        ) from e
    if not callable(obj):
        raise ValueError(f"The imported object is not callable: '{name}'")
    return obj


def resolve_obs_groups(obs, obs_groups: dict, default_sets: list) -> dict:
    """Validate the observation-set configuration and fill in missing default sets.

    Same contract as rsl_rl/utils/utils.py:202-304: 'policy' must be configured (or present as an
    observation group, with a warning); empty sets and unknown groups raise ValueError; each missing
    default set takes the observation group of the same name if there is one, else a copy of the
    'policy' set (with a warning).
    """
    if "policy" not in obs_groups:
        if "policy" not in obs:
            raise ValueError(
                "The observation configuration dictionary 'obs_groups' must contain the 'policy' key."
                f" Found keys: {list(obs_groups.keys())}"
            )
        obs_groups["policy"] = ["policy"]
        warnings.warn(
            "The observation configuration dictionary 'obs_groups' must contain the 'policy' key. As an"
            " observation group with the name 'policy' was found, this is assumed to be the observation set."
            " Consider adding the 'policy' key to the 'obs_groups' dictionary for clarity. This behavior will"
            " be removed in a future version."
        )

    for set_name, groups in obs_groups.items():
        if len(groups) == 0:
            msg = f"The '{set_name}' key in the 'obs_groups' dictionary can not be an empty list."
            if set_name in default_sets:
                if set_name in obs:
                    msg += f" Consider removing the key to default to the observation '{set_name}' from the environment."
                else:
                    msg += " Consider removing the key to default to the observations used for the 'policy' set."
            raise ValueError(msg)
        for group in groups:
            if group not in obs:
                raise ValueError(
                    f"Observation '{group}' in observation set '{set_name}' not found in the observations from the"
                    f" environment. Available observations from the environment: {list(obs.keys())}"
                )

    for name in default_sets:
        if name in obs_groups:
            continue
        if name in obs:
            obs_groups[name] = [name]
            warnings.warn(
                f"The observation configuration dictionary 'obs_groups' must contain the '{name}' key. As an"
                f" observation group with the name '{name}' was found, this is assumed to be the observation set."
                f" Consider adding the '{name}' key to the 'obs_groups' dictionary for clarity. This behavior will"
                " be removed in a future version."
            )
        else:
            obs_groups[name] = list(obs_groups["policy"])
            warnings.warn(
                f"The observation configuration dictionary 'obs_groups' must contain the '{name}' key. As the"
                f" configuration for '{name}' is missing, the observations from the 'policy' set are used. Consider"
                f" adding the '{name}' key to the 'obs_groups' dictionary for clarity. This behavior will be removed"
                " in a future version."
            )

    print("-" * 80)
    print("Resolved observation sets: ")
    for set_name, groups in obs_groups.items():
        print("\t", set_name, ": ", groups)
    print("-" * 80)
    return obs_groups


def store_code_state(logdir, repositories) -> list:
    """Write `git status` + `git diff HEAD` of each repository once into <logdir>/git/<repo>.diff
    (utils.py:144-169), using the git CLI."""
    if logdir is None:
        return []
    git_dir = os.path.join(logdir, "git")
    os.makedirs(git_dir, exist_ok=True)
    paths = []
    for repo_file in repositories:
        start = repo_file if os.path.isdir(repo_file) else os.path.dirname(os.path.abspath(repo_file))
        try:
            top = subprocess.run(["git", "-C", start, "rev-parse", "--show-toplevel"], capture_output=True,
                                 text=True, check=True).stdout.strip()
        except (OSError, subprocess.CalledProcessError):
            print(f"Could not find git repository in {repo_file}. Skipping.")
            continue
        name = pathlib.Path(top).name
        diff_file = os.path.join(git_dir, f"{name}.diff")
        if os.path.isfile(diff_file):
            continue
        status = subprocess.run(["git", "-C", top, "status"], capture_output=True, text=True).stdout
        diff = subprocess.run(["git", "-C", top, "diff", "HEAD"], capture_output=True, text=True).stdout
        print(f"Storing git diff for '{name}' in: {diff_file}")
        with open(diff_file, "x", encoding="utf-8") as f:
            f.write(f"--- git status ---\n{status} \n\n\n--- git diff ---\n{diff}")
        paths.append(diff_file)
    return paths
