"""Host time of PPO.update (ppo.py:178-422) on the bench's configuration: wall time per update, the GPU time of its
kernels (HIP events), and a cProfile of the same updates (top functions by own time, plus the time spent waiting in the
one read-back) -- whether the update is launch-bound at a given env count.

    python scripts/update_host_profile.py --num-envs 16384 --iters 5 --out gpurun_out/update_host.json
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
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/update_host.json")
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

    def rollout():
        nonlocal obs
        with torch.inference_mode(), fused_mlp.frozen_weights():
            for _ in range(24):
                actions = alg.act(obs)
                obs, rewards, dones, extras = env.step(actions.to(env.device))
                alg.process_env_step(obs, rewards, dones, extras)
            alg.compute_returns(obs)

    walls, gpus, enq = [], [], []
    pr = cProfile.Profile()
    for it in range(a.iters + 1):
        rollout()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        prof = it == a.iters
        e0.record()
        t0 = time.perf_counter()
        if prof:
            pr.enable()
        alg.update()
        if prof:
            pr.disable()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        if not prof:
            walls.append((t1 - t0) * 1e3)
            gpus.append(e0.elapsed_time(e1))
    sio = io.StringIO()
    st = pstats.Stats(pr, stream=sio)
    st.sort_stats("tottime").print_stats(25)
    waits = sum(v[3] for k, v in st.stats.items() if k[2] in ("synchronize", "item", "cpu", "tolist")
                or "method 'cpu'" in k[2] or "method 'item'" in k[2] or "method 'tolist'" in k[2])
    res = {"num_envs": a.num_envs, "update_wall_ms": [round(x, 2) for x in walls],
           "update_gpu_event_ms": [round(x, 2) for x in gpus], "profiled_update_wait_s": round(waits, 4),
           "profiled_update_total_s": round(st.total_tt, 4), "cprofile_tottime_top25": sio.getvalue()}
    print(json.dumps({k: v for k, v in res.items() if k != "cprofile_tottime_top25"}), flush=True)
    print(sio.getvalue(), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
