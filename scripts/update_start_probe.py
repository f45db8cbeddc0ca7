"""Host time of the update's first mini-batch on the bench's configuration (the GPU idles from the end of
compute_returns to the first MLP launch): per-call host microseconds of the pieces between PPO.update's entry and the
first mini-batch's launches (draw_permutation, _start_prefetch, the gather, the first-mini-batch setup), the median over
several updates.

    python scripts/update_start_probe.py --num-envs 16384 --iters 6 --out gpurun_out/update_start.json
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import statistics
import sys
import time
from collections import defaultdict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--out", default="gpurun_out/update_start.json")
    a = ap.parse_args()

    import bench
    from rsl_rl_amd import kernels
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.networks import fused_mlp
    from rsl_rl_amd.runners import OnPolicyRunner
    from rsl_rl_amd.storage import rollout_storage as rs

    dev = "cuda:0"
    bargs = argparse.Namespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    torch.manual_seed(1)
    env = SyntheticVecEnv(a.num_envs, 48, 12, device=dev, seed=0)
    with contextlib.redirect_stdout(sys.stderr):
        runner = OnPolicyRunner(env, bench.train_cfg(bargs), log_dir=None, device=dev)
        runner.learn(2)
    alg = runner.alg
    times = defaultdict(list)
    marks = {}

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*args, **kw):
            t = time.perf_counter()
            try:
                return f(*args, **kw)
            finally:
                times[label].append((time.perf_counter() - t) * 1e6)
        setattr(obj, name, g)

    from rsl_rl_amd.algorithms import ppo as ppo_mod
    from rsl_rl_amd.modules import actor_critic as ac_mod

    wrap(ac_mod.ActorCritic, "manual_update_ok", "manual_update_ok")
    wrap(ppo_mod.PPO, "grad_arena", "grad_arena")
    wrap(ac_mod.ActorCritic, "train_forward", "train_forward")
    wrap(fused_mlp, "train_forward_pair", "train_forward_pair")
    ac_mod.fused_mlp.train_forward_pair = fused_mlp.train_forward_pair
    wrap(rs.RolloutStorage, "draw_permutation", "draw_permutation")
    wrap(rs.RolloutStorage, "_start_prefetch", "start_prefetch")
    wrap(rs.RolloutStorage, "_packed_buffers", "packed_buffers")
    wrap(kernels, "gather_records_side", "gather_records_side")
    rs.kernels.gather_records_side = kernels.gather_records_side
    orig_bimages = fused_mlp.bimages

    def bimages(specs):
        if "first_bimage" not in marks:
            marks["first_bimage"] = time.perf_counter()
        t = time.perf_counter()
        r = orig_bimages(specs)
        times["bimages"].append((time.perf_counter() - t) * 1e6)
        return r
    fused_mlp.bimages = bimages
    orig_fwd_pair = fused_mlp.linear_fwd_pair

    def linear_fwd_pair(*a, **k):
        if "first_mlp" not in marks:
            marks["first_mlp"] = time.perf_counter()
        return orig_fwd_pair(*a, **k)
    fused_mlp.linear_fwd_pair = linear_fwd_pair

    obs = env.get_observations()
    for it in range(a.iters):
        with torch.inference_mode(), fused_mlp.frozen_weights():
            for _ in range(24):
                actions = alg.act(obs)
                obs, rewards, dones, extras = env.step(actions.to(env.device))
                alg.process_env_step(obs, rewards, dones, extras)
            alg.compute_returns(obs)
        torch.cuda.synchronize()
        marks.clear()
        t0 = time.perf_counter()
        alg.update()
        if "first_bimage" in marks:
            times["update_entry_to_first_bimage"].append((marks["first_bimage"] - t0) * 1e6)
        if "first_mlp" in marks:
            times["update_entry_to_first_mlp_launch"].append((marks["first_mlp"] - t0) * 1e6)
    res = {k: {"median_us": round(statistics.median(v[1:] if len(v) > 2 else v), 1), "n": len(v)}
           for k, v in times.items()}
    res["num_envs"] = a.num_envs
    print(json.dumps(res), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
