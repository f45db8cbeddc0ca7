"""Host-side profile of one training iteration at C3 (torch.profiler, CPU activities only): which Python/ATen calls
the launch thread spends its time in during the rollout and the update.  Diagnostic, not part of the bench.

    python scripts/rollout_host_profile.py > gpurun_out/host_profile.txt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rsl_rl_amd.env import SyntheticVecEnv  # noqa: E402
from rsl_rl_amd.runners import OnPolicyRunner  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    import types
    args = types.SimpleNamespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    torch.manual_seed(1)
    env = SyntheticVecEnv(65536, args.num_obs, args.num_actions, device=dev)
    runner = OnPolicyRunner(env, bench.train_cfg(args), log_dir=None, device=dev)
    runner.learn(3)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        runner.learn(1)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))


if __name__ == "__main__":
    main()
