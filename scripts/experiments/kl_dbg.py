import os, sys, torch
sys.path.insert(0, os.getcwd())
import rsl_rl_amd.algorithms.ppo as P
orig = P.adapt_learning_rate_device
def wrap(lr, kl, d):
    print("KL", kl.item(), "lr", lr.item(), flush=True)
    return orig(lr, kl, d)
P.adapt_learning_rate_device = wrap
import pytest
sys.exit(pytest.main(["-x", "-q", "-s", "tests/test_gpu_update.py::test_update_c1_matches_reference"]))
