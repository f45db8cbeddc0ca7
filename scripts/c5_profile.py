"""C5 (C3 + RND) iterations for a rocprofv3 kernel trace: python scripts/c5_profile.py [iters] [--no-rnd]."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rsl_rl_amd.env import SyntheticVecEnv  # noqa: E402
from rsl_rl_amd.runners import OnPolicyRunner  # noqa: E402


class A:
    num_steps_per_env, num_obs, num_actions, hidden, layers = 24, 48, 12, 256, 3


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
    rnd = "--no-rnd" not in sys.argv
    torch.manual_seed(1)
    env = SyntheticVecEnv(65536, 48, 12, device="cuda:0", seed=0)
    with contextlib.redirect_stdout(sys.stderr):
        runner = OnPolicyRunner(env, bench.train_cfg(A, rnd=rnd), log_dir=None, device="cuda:0")
        runner.learn(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.learn(iters)
        torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / iters
    print({"ms_per_iter": round(el * 1e3, 3), "rnd": rnd, "fused_rnd": getattr(runner.alg, "_rnd_adam", None) is not None,
           "phases": runner.last_iteration_stats})


if __name__ == "__main__":
    main()
