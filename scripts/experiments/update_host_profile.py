"""Host-side cost of one PPO.update() at a given env count: wall time of the call (host issue, GPU behind) and a
cProfile of it sorted by own time.  Diagnostic: python scripts/update_host_profile.py [num_envs]"""
import cProfile
import io
import os
import pstats
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rsl_rl_amd.env import SyntheticVecEnv  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402
from rsl_rl_amd.runners import OnPolicyRunner  # noqa: E402


def fill(runner, env, obs):
    alg = runner.alg
    with torch.inference_mode(), fused_mlp.frozen_weights():
        for _ in range(24):
            actions = alg.act(obs)
            obs, rewards, dones, extras = env.step(actions)
            alg.process_env_step(obs, rewards, dones, extras)
        alg.compute_returns(obs)
    return obs


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    args = types.SimpleNamespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    env = SyntheticVecEnv(n, 48, 12, device=dev)
    runner = OnPolicyRunner(env, bench.train_cfg(args), log_dir=None, device=dev)
    runner.learn(2)
    obs = env.get_observations().to(dev)
    obs = fill(runner, env, obs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.alg.update()  # ends with one read-back of the loss statistics (waits for the GPU)
    t1 = time.perf_counter()
    print(f"update wall {1e3 * (t1 - t0):.2f} ms")
    obs = fill(runner, env, obs)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    runner.alg.update()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
