"""Host-side cost of the rollout at C3: cProfile of the launch thread over one iteration's 24 env steps (after
warm-up), and the host issue time per step next to the GPU time per step.  Diagnostic, not part of the bench.

    python scripts/rollout_host_profile.py > gpurun_out/host_profile.txt
"""
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


def main():
    dev = torch.device("cuda:0")
    args = types.SimpleNamespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    torch.manual_seed(1)
    env = SyntheticVecEnv(int(os.environ.get("HP_ENVS", 65536)), args.num_obs, args.num_actions, device=dev)
    runner = OnPolicyRunner(env, bench.train_cfg(args), log_dir=None, device=dev)
    runner.learn(3)
    torch.cuda.synchronize()
    alg = runner.alg
    obs = env.get_observations().to(dev)

    def rollout(n):
        nonlocal obs
        with torch.inference_mode(), fused_mlp.frozen_weights():
            for _ in range(n):
                actions = alg.act(obs)
                obs, rewards, dones, extras = env.step(actions)
                alg.process_env_step(obs, rewards, dones, extras)
        alg.storage.clear()

    # host issue time vs GPU time per step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rollout(24)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e6 * (t1 - t0) / 24:.1f} us/step, until GPU done {1e6 * (t2 - t0) / 24:.1f} us/step")
    # the policy half alone (act + process_env_step on a fixed env output): host issue per step
    with torch.inference_mode(), fused_mlp.frozen_weights():
        o2, r2, d2, e2 = env.step(alg.act(obs))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.inference_mode(), fused_mlp.frozen_weights():
        for _ in range(24):
            alg.act(obs)
            alg.process_env_step(o2, r2, d2, e2)
    t1 = time.perf_counter()
    alg.storage.clear()
    torch.cuda.synchronize()
    print(f"policy half host issue {1e6 * (t1 - t0) / 24:.1f} us/step")
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    rollout(24)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
