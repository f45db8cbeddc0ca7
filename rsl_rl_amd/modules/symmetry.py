"""Symmetry config resolution (rsl_rl/modules/symmetry.py:9-24)."""

from __future__ import annotations


def resolve_symmetry_config(alg_cfg, env):
    """Inject the environment into symmetry_cfg["_env"] for the augmentation function."""
    if alg_cfg.get("symmetry_cfg") is not None:
        alg_cfg["symmetry_cfg"]["_env"] = env
    return alg_cfg
