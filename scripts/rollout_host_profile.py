"""Host time of the rollout loop (on_policy_runner.py:104-109: act, env.step, process_env_step) on the bench's
configuration: per-call host microseconds of the three calls over many steps (the GPU queue kept full), the GPU time per
step from HIP events, and a cProfile of the same steps (top functions by own time).

    python scripts/rollout_host_profile.py --num-envs 16384 --steps 240 --out gpurun_out/rollout_host.json
"""

from __future__ import annotations

import argparse
import contextlib
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--out", default="gpurun_out/rollout_host.json")
    a = ap.parse_args()

    import bench
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.networks import fused_mlp
    from rsl_rl_amd.runners import OnPolicyRunner

    dev = "cuda:0"
    bargs = argparse.Namespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    torch.manual_seed(1)
    env = SyntheticVecEnv(a.num_envs, 48, 12, device=dev, seed=0)
    with contextlib.redirect_stdout(sys.stderr):
        runner = OnPolicyRunner(env, bench.train_cfg(bargs), log_dir=None, device=dev)
        runner.learn(2)
    alg = runner.alg
    obs = env.get_observations()
    obs = obs.to(dev) if hasattr(obs, "to") else obs
    T = 24

    def steps(n, prof=None):
        tt = [0.0, 0.0, 0.0]
        nonlocal obs
        with torch.inference_mode(), fused_mlp.frozen_weights():
            for k in range(n):
                if k % T == 0:
                    alg.storage.clear()
                t0 = time.perf_counter()
                actions = alg.act(obs)
                t1 = time.perf_counter()
                obs, rewards, dones, extras = env.step(actions.to(env.device))
                t2 = time.perf_counter()
                alg.process_env_step(obs, rewards, dones, extras)
                t3 = time.perf_counter()
                tt[0] += t1 - t0
                tt[1] += t2 - t1
                tt[2] += t3 - t2
        return tt

    steps(2 * T)  # warm (graph capture)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    tt = steps(a.steps)
    host = time.perf_counter() - h0
    e1.record()
    torch.cuda.synchronize()
    gpu_us = e0.elapsed_time(e1) * 1e3 / a.steps
    res = {"num_envs": a.num_envs, "steps": a.steps, "host_us_per_step": round(host * 1e6 / a.steps, 2),
           "gpu_us_per_step_wall": round(gpu_us, 2),
           "act_us": round(tt[0] * 1e6 / a.steps, 2), "env_step_us": round(tt[1] * 1e6 / a.steps, 2),
           "process_env_step_us": round(tt[2] * 1e6 / a.steps, 2)}
    print(json.dumps(res), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    steps(a.steps)
    pr.disable()
    torch.cuda.synchronize()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(30)
    res["cprofile_tottime_top30"] = sio.getvalue()
    print(sio.getvalue(), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
