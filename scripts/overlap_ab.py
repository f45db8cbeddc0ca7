"""What the update's gradient collective costs on RCCL, measured at world 1.

A world-1 "nccl" (RCCL) group still launches RCCL's all-reduce kernel for every call, so forcing PPO's multi-GPU
path at world 1 shows what the collective -- and the round-5 early-prefix overlap, an asynchronous all-reduce of the
upper layers' gradients issued while the first layers' backward still runs -- cost the one-workgroup-per-CU kernels
that co-run with it.  Modes, alternated in one process (ppo.py:446-456, :503-508):
  none     is_multi_gpu False: no collective (the N = 1 bench path)
  single   one SUM all-reduce of the arena + KL per mini-batch after the backward (RSLRL_OVERLAP_ALLREDUCE=0)
  overlap  the early prefix asynchronously during the backward, the rest after it (the round-5 default)

    python scripts/overlap_ab.py --num-envs 65536 16384 --iters 10 --rounds 3 --out gpurun_out/overlap_ab.json
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def set_mode(alg, mode):
    alg.is_multi_gpu = mode != "none"
    alg.gpu_world_size = 1
    alg.gpu_global_rank = 0
    os.environ["RSLRL_OVERLAP_ALLREDUCE"] = "1" if mode == "overlap" else "0"
    alg._arena = None  # rebuilt at the next update with (or without) the early prefix


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, nargs="+", default=[65536, 16384])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", nargs="+", default=["none", "single", "overlap"])
    ap.add_argument("--out", default="gpurun_out/overlap_ab.json")
    a = ap.parse_args()

    import bench
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.runners import OnPolicyRunner

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    bargs = argparse.Namespace(num_steps_per_env=24, num_obs=48, num_actions=12, hidden=256, layers=3)
    out = {"note": __doc__.strip().splitlines()[0], "runs": []}
    for n in a.num_envs:
        torch.manual_seed(1)
        env = SyntheticVecEnv(n, 48, 12, device="cuda:0", seed=0)
        with contextlib.redirect_stdout(sys.stderr):
            runner = OnPolicyRunner(env, bench.train_cfg(bargs), log_dir=None, device="cuda:0")
            for mode in a.modes:  # warm every mode's arena layout and RCCL's communicator
                set_mode(runner.alg, mode)
                runner.learn(1)
        res = {m: [] for m in a.modes}
        for r in range(a.rounds):
            for mode in (a.modes if r % 2 == 0 else a.modes[::-1]):
                set_mode(runner.alg, mode)
                with contextlib.redirect_stdout(sys.stderr):
                    runner.learn(1)  # the arena is rebuilt here
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    runner.learn(a.iters)
                    torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / a.iters * 1e3
                res[mode].append(ms)
                print(json.dumps({"num_envs": n, "round": r, "mode": mode, "ms_per_iter": round(ms, 3)}), flush=True)
        summ = {m: {"ms_per_iter": [round(x, 3) for x in v], "median": round(statistics.median(v), 3),
                    "env_steps_per_s": round(24 * n / (statistics.median(v) * 1e-3), 1)} for m, v in res.items()}
        base = summ.get("none", {}).get("median")
        if base:
            for m in summ:
                summ[m]["vs_none"] = round(summ[m]["median"] / base - 1.0, 4)
        out["runs"].append({"num_envs": n, "iters": a.iters, "rounds": a.rounds, "modes": summ})
        print(json.dumps(out["runs"][-1]), flush=True)
        del runner, env
        torch.cuda.empty_cache()
    dist.destroy_process_group()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
