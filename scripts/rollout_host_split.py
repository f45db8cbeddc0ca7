"""Host issue time per rollout step, split into act() / env.step() / process_env_step() (no profiler overhead;
the GPU runs behind).  Diagnostic: python scripts/rollout_host_split.py [num_envs]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rsl_rl_amd.env import SyntheticVecEnv  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402
from rsl_rl_amd.runners import OnPolicyRunner  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    args = types.SimpleNamespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    env = SyntheticVecEnv(n, 48, 12, device=dev)
    runner = OnPolicyRunner(env, bench.train_cfg(args), log_dir=None, device=dev)
    runner.learn(2)
    alg = runner.alg
    obs = env.get_observations().to(dev)
    tot = {"act": 0.0, "env": 0.0, "record": 0.0}
    reps = 5
    for _ in range(reps):
        torch.cuda.synchronize()
        with torch.inference_mode(), fused_mlp.frozen_weights():
            for _ in range(24):
                t0 = time.perf_counter()
                actions = alg.act(obs)
                t1 = time.perf_counter()
                obs, rewards, dones, extras = env.step(actions)
                t2 = time.perf_counter()
                alg.process_env_step(obs, rewards, dones, extras)
                t3 = time.perf_counter()
                tot["act"] += t1 - t0
                tot["env"] += t2 - t1
                tot["record"] += t3 - t2
        alg.storage.clear()
    print({k: round(1e6 * v / (24 * reps), 1) for k, v in tot.items()}, "us per step (host issue)")


if __name__ == "__main__":
    main()
