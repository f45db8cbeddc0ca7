"""PPO env-steps/sec (rollout + GAE + update) on MI355X -- BASELINE.json's headline metric.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: starts its own N ranks via torch.distributed.run)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Workload.  N=1 (the metric's configuration, C3 = BASELINE.json configs[2]): 65536 synthetic envs, T=24 steps/env,
obs 48, 12 actions, actor/critic MLP 3x256 ELU, PPO defaults (E=5 epochs x M=4 mini-batches, adaptive KL lr).
N>1 (C4 = configs[3]): 131072 envs in total, partitioned over the ranks (16384 per GPU at N=8) -- the envs shard,
every rank owns its slice, its storage and its permutation; gradients (+ the KL) are averaged by ONE RCCL
all-reduce per mini-batch ("scaling": "strong": the total work is fixed as N grows).  --global-num-envs sets the
total, --num-envs a fixed per-GPU count instead (weak scaling).  One "step" = one OnPolicyRunner iteration:
T rollout steps + compute_returns + update.  `value` = T * total envs / (max over ranks of the timed seconds).

The MLP GEMMs run on the x6 split-bf16 kernels (fp32 operands as three bf16 planes, 24 significant bits, six
products, fp32 accumulation: fp32-faithful); `extra_configs` adds C5 (RND), the exact-fp32 MFMA kernels, the
reduced-precision h3 mode (labelled as such) and the C4 total on one GPU (the strong-scaling base point).

Extra fields: `roofline` for the dominant hot-path kernel (algorithmic bytes / live HIP-event duration on its
stream, against 8 TB/s), `hot_path` (per-kernel times per iteration), `roofline_mlp`, and `cpu_baseline` (the
reference's iteration restated in torch-CPU ops, oracle/torch_cpu_ppo.py, on the box's host cores, rank 0, N=1
only, bounded samples).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA at 2.4 GHz (MI355X_MICROARCH.md)
X6_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6  # fp32-equivalent peak of the 6-product split-bf16 GEMMs
H3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3  # ... of the 3-product split-fp16 GEMMs (fp16 MFMA = bf16 rate)
FP32_MFMA_PEAK_TFLOPS = 157.3
HOT_PATH = ("compute_returns", "record_fill_slot", "gather_rows", "ppo_loss", "rollout_record", "rnd_update")
C3_ENVS = 65536  # BASELINE.json configs[2] (N=1 headline)
with open(os.path.join(ROOT, "BASELINE.json")) as _f:
    BASELINE_METRIC = json.load(_f)["metric"]
C4_ENVS = 131072  # BASELINE.json configs[3]: the total partitioned over the ranks
# per-launch HBM traffic of the hot-path kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this same
# bench command (scripts/pmc_summary.py; raw counters next to it).  PMC passes serialise and slow the
# run, so they are collected separately and the committed summary is reported here.
# One summary per profiled workload (scripts/pmc_summary.py --num-envs): bench.py reports `traffic` only from the file
# whose recorded workload (envs per GPU, T) is the run's own, else null -- per-launch traffic does not carry over
# between workloads (round 5 quoted C3's for every workload).
PMC_TRAFFIC_GLOB = os.path.join(ROOT, "profiles", "r6_pmc_traffic*.json")
# the MLP GEMM pairs' counters (scripts/mlp_pmc.sh + scripts/mlp_pmc_summary.py over scripts/mlp_pair_probe.py at C3's
# 393,216-row mini-batch): FETCH_SIZE / WRITE_SIZE corrected by factors calibrated on the box in each kernel's own
# access pattern (scripts/pmc_pattern_probe.hip), plus clock and MFMA-pipe utilisation from the SQ counters
MLP_PMC_FILE = os.path.join(ROOT, "profiles", "r5_mlp_pmc.json")
MLP_PMC_NAMES = {"linear_hidden_bwd_pair[M=393216,N=256,K=256]": "x6_hidden_bwd_pair",
                 "linear_dgrad_pair[M=393216,Nred=256,K=256]": "x6_dgrad_pair_w4",
                 "linear_fwd_pair[M=393216,K=256,N=256]": "x6_fwd_stream_pair",
                 "linear_wgrad_pair[M=393216,N=256,K=256]": "x6_wgrad_pair"}


# hot-path timer names -> PMC summary names (scripts/pmc_summary.py SHORT)
PMC_NAMES = {"compute_returns": "compute_returns_one_launch"}


def mlp_pmc(kernel):
    try:
        with open(MLP_PMC_FILE) as f:
            k = json.load(f)["kernels"].get(MLP_PMC_NAMES.get(kernel, ""))
    except (OSError, ValueError, KeyError):
        return None
    if not k:
        return None
    return {"traffic_bytes": k.get("traffic_bytes"), "traffic_over_algorithmic": k.get("traffic_over_algorithmic"),
            "clock_GHz": k.get("clock_GHz"), "mfma_pipe_util": k.get("mfma_pipe_util"),
            "source": os.path.relpath(MLP_PMC_FILE, ROOT)}


def pmc_traffic(kernel, num_envs, T):
    """(traffic bytes per launch, source) of `kernel` from the PMC summary of this workload, or (None, reason)."""
    import glob
    for path in sorted(glob.glob(PMC_TRAFFIC_GLOB)):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        w = d.get("workload") or {}
        if w.get("num_envs_per_gpu") == num_envs and w.get("num_steps_per_env") == T:
            k = d.get("kernels", {}).get(kernel)
            src = os.path.relpath(path, ROOT)
            return (k["traffic_bytes"], src) if k else (None, f"{src} has no {kernel} entry")
    return None, f"no PMC summary for {num_envs} envs x T={T} (profiles/r6_pmc_traffic*.json)"


def train_cfg(args, rnd=False):
    hidden = [args.hidden] * args.layers
    cfg = {
        "num_steps_per_env": args.num_steps_per_env,
        "save_interval": 10**9,
        "obs_groups": {"policy": ["policy"], "critic": ["policy"]},
        "policy": {"class_name": "ActorCritic", "activation": "elu", "actor_hidden_dims": hidden,
                   "critic_hidden_dims": hidden, "init_noise_std": 1.0, "noise_std_type": "scalar",
                   "actor_obs_normalization": False, "critic_obs_normalization": False},
        "algorithm": {"class_name": "PPO", "learning_rate": 1e-3, "num_learning_epochs": 5, "num_mini_batches": 4,
                      "schedule": "adaptive", "value_loss_coef": 1.0, "clip_param": 0.2,
                      "use_clipped_value_loss": True, "desired_kl": 0.01, "entropy_coef": 0.01, "gamma": 0.99,
                      "lam": 0.95, "max_grad_norm": 1.0, "normalize_advantage_per_mini_batch": False},
    }
    if rnd:  # config C5: RND weight 1.0 (x step_dt), 1 output, hidden [-1], no normalisation
        cfg["obs_groups"]["rnd_state"] = ["policy"]
        cfg["algorithm"]["rnd_cfg"] = {"weight": 1.0, "num_outputs": 1, "predictor_hidden_dims": [-1],
                                       "target_hidden_dims": [-1], "learning_rate": 1e-3,
                                       "state_normalization": False, "reward_normalization": False}
    return cfg


def time_runner(args, device, rank, *, rnd=False, steps=5, warmup=2, num_envs=None):
    """Iterations/s of a fresh runner (for the secondary configurations; world size 1 only)."""
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.runners import OnPolicyRunner

    n = num_envs or args.num_envs_local
    torch.manual_seed(1)
    env = SyntheticVecEnv(n, args.num_obs, args.num_actions, device=device, seed=rank)
    with contextlib.redirect_stdout(sys.stderr):
        runner = OnPolicyRunner(env, train_cfg(args, rnd=rnd), log_dir=None, device=device)
        runner.learn(warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.learn(steps)
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    stats = {k: round(v, 4) for k, v in runner.last_iteration_stats.items() if k != "loss_dict"}
    del runner, env
    torch.cuda.empty_cache()
    T = args.num_steps_per_env
    return {"value": round(T * n * steps / el, 1), "unit": "env-steps/s", "steps": steps, "warmup": warmup,
            "num_envs": n, "ms_per_step": round(el / steps * 1e3, 3), "phases_last_iter": stats}


def _cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 CPU quota when one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            n = max(1, min(n, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args):
    """The reference's PPO iteration in torch-CPU ops (oracle/torch_cpu_ppo.py) on every CPU this process may use:
    a bounded sample of the C3 iteration at its full size (N 65536: the whole rollout and compute_returns, then
    `--cpu-mini-batches` of the 20 update mini-batches, the update extrapolated from them) = value, and one whole
    C2 iteration (N 4096) for reference.  scripts/ref_cpu_timing.py times the reference's own iteration next to this
    port on the build host (the port runs ~1.2x faster than the reference there: the baseline is not understated)."""
    from oracle import torch_cpu_ppo

    share = _cpu_share()
    # torch's CPU GEMMs do not always run fastest on every CPU of a throttled share: take the faster of the share
    # and half of it on a short C2-sized probe (the thread count used is what `cores` reports)
    probe = {}
    for th in sorted({share, max(1, share // 2)}, reverse=True):
        probe[th] = torch_cpu_ppo.time_iterations(4096, args.num_obs, args.num_actions, T=args.num_steps_per_env,
                                                  iters=1, warmup=0, threads=th)[0]
    threads = max(probe, key=probe.get)
    out = {}
    rate, secs, parts = torch_cpu_ppo.time_iterations(4096, args.num_obs, args.num_actions, T=args.num_steps_per_env,
                                                      iters=1, warmup=1, threads=threads)
    out["C2"] = {"env_steps_per_s": round(rate, 1), "num_envs": 4096, "timed_seconds": round(secs, 2),
                 "update_env_steps_per_s": round(parts["update_env_steps_per_s"], 1), "phase_seconds": parts["seconds"],
                 # the C3 sample's extrapolation rule applied to this whole C2 iteration's own mini-batch times
                 "extrapolation_check": parts["extrapolation_check"]}
    n = args.num_envs_local
    rate, secs, parts = torch_cpu_ppo.time_full_size_sample(n, args.num_obs, args.num_actions,
                                                            T=args.num_steps_per_env,
                                                            mini_batches=args.cpu_mini_batches, threads=threads)
    out["C3_full_size_sample"] = {"env_steps_per_s": round(rate, 1), "num_envs": n, "timed_seconds": round(secs, 2),
                                  "update_env_steps_per_s": round(parts["update_env_steps_per_s"], 1),
                                  "phase_seconds": parts["seconds"]}
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    big = out["C3_full_size_sample"]
    return {
        "value": big["env_steps_per_s"],
        "unit": "env-steps/s",
        "cores": threads,
        "kind": "port",
        "update_env_steps_per_s": big["update_env_steps_per_s"],
        "samples": out,
        "thread_probe_c2_env_steps_per_s": {str(k): round(v, 1) for k, v in probe.items()},
        "extrapolation_error_on_whole_c2_update": out["C2"]["extrapolation_check"].get(
            f"first_{args.cpu_mini_batches}", {}).get("rel_error"),
        "cpu_share": share,
        "sample": f"the reference's algorithm in torch-CPU ops (oracle/torch_cpu_ppo.py: rollout, compute_returns loop, "
                  f"randperm + per-mini-batch gathers, Normal log-prob/entropy/KL, clipped losses, autograd, "
                  f"clip_grad_norm_, Adam) at the bench workload's full size N={n}, T={args.num_steps_per_env}, obs "
                  f"{args.num_obs}, act {args.num_actions}, 3x256 MLP: the whole rollout + compute_returns timed, then "
                  f"{args.cpu_mini_batches} of the 20 update mini-batches, the update extrapolated as first + 19 x "
                  f"mean(rest) (value); plus one whole C2 iteration (N 4096), on which the same extrapolation is checked "
                  f"against its measured update (extrapolation_error_on_whole_c2_update); {threads} threads (the faster of the "
                  f"{share}-CPU affinity/cgroup share and half of it on a C2 probe); CPU: {model}",
    }


def hot_path_summary(hot, hot_ms, mlp, T, N):
    """SURVEY.md §8(a)'s hot path per iteration: the stand-alone kernels (rollout record, compute_returns, record
    gather; marker spans of the timed region) and, since round 4, the PPO loss, which runs inside the actor's fused head
    launch (last hidden layer + output layer + loss + output-layer backward): that whole launch is counted
    for it (its event time from the MLP-timed iteration), so the figure with it is an upper bound on the loss's share."""
    out = {"kernels": hot, "ms_per_step": round(hot_ms, 4),
           "env_steps_per_s": round(T * N / (hot_ms * 1e-3), 1) if hot_ms else None,
           "ppo_loss": "inside linear_actor_head (not a stand-alone launch on the default path); see "
                       "ms_per_step_with_actor_head"}
    head = [k for k in mlp if k.startswith("linear_actor_head")]
    if head:
        h = mlp[head[0]]
        out["actor_head_launch"] = {"kernel": head[0], "mean_us": h["mean_us"], "ms_per_step": h["ms_per_step"],
                                    "launches_per_step": h["launches_per_step"]}
        with_head = hot_ms + h["ms_per_step"]
        out["ms_per_step_with_actor_head"] = round(with_head, 4)
        out["env_steps_per_s_with_actor_head"] = round(T * N / (with_head * 1e-3), 1)
    else:  # the loss runs as its own kernel (another shape / std type): it is one of `kernels`
        out["ppo_loss"] = "stand-alone ppo_loss launches (in kernels)"
    return out


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """One process per GPU for `python bench.py --gpus N` run without a launcher: torch.distributed.run as a child
    process (one node, N ranks, rendezvous on 127.0.0.1) re-running this script with the same arguments; each rank
    reads RANK / LOCAL_RANK / WORLD_SIZE and takes cuda:LOCAL_RANK.  Returns the launcher's exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the box's driver has no legacy IPC)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-envs", type=int, default=None,
                    help="environments per GPU (weak scaling); default: --global-num-envs split over the ranks")
    ap.add_argument("--global-num-envs", type=int, default=None,
                    help=f"environments in total, partitioned over the ranks (strong scaling); default {C3_ENVS} "
                         f"on one GPU (C3), {C4_ENVS} over N > 1 GPUs (C4)")
    ap.add_argument("--num-steps-per-env", type=int, default=24)
    ap.add_argument("--num-obs", type=int, default=48)
    ap.add_argument("--num-actions", type=int, default=12)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--cpu-mini-batches", type=int, default=3,
                    help="update mini-batches the CPU baseline times at full size (the rest are extrapolated)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary configurations (C5, f32 / h3 GEMMs, C4 total on one GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: start the N ranks here (this process has not touched the GPU)
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("RSLRL_BENCH_RANK_ENV_ONLY") == "1":  # launcher check (tests/test_bench_launch.py): no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                         "MASTER_ADDR", "MASTER_PORT")}), flush=True)
        return
    visible = torch.cuda.device_count()  # does not initialise the GPU on this image
    # test-only (tests/test_bench_launch.py): every rank on cuda:0 over gloo, so the N > 1 line runs on one GPU
    one_device = world > 1 and os.environ.get("RSLRL_TEST_ONE_DEVICE") == "1"
    dev_index = 0 if one_device else local_rank
    if dev_index >= visible:
        raise SystemExit(f"bench.py rank {rank}: --gpus {world} needs {world} GPUs on this node, {visible} visible")
    torch.cuda.set_device(dev_index)
    device = f"cuda:{dev_index}"
    if args.num_envs is not None:
        if args.global_num_envs is not None:
            raise SystemExit("--num-envs (per GPU) and --global-num-envs (total) are exclusive")
        args.num_envs_local, scaling = args.num_envs, "weak"
        total = args.num_envs * world
    else:
        total = args.global_num_envs or (C3_ENVS if world == 1 else C4_ENVS)
        if total % world:
            raise SystemExit(f"--global-num-envs {total} does not split evenly over {world} ranks")
        args.num_envs_local, scaling = total // world, "strong"

    from rsl_rl_amd import kernels
    from rsl_rl_amd.env import SyntheticVecEnv
    from rsl_rl_amd.runners import OnPolicyRunner

    torch.manual_seed(1)  # policy init; the env stream is seeded per rank
    env = SyntheticVecEnv(args.num_envs_local, args.num_obs, args.num_actions, device=device, seed=rank)
    with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the result line
        runner = OnPolicyRunner(env, train_cfg(args), log_dir=None, device=device)  # inits RCCL when world > 1

    def barrier():
        if world > 1:
            dist.barrier()

    with contextlib.redirect_stdout(sys.stderr):  # learn() prints (rank sync messages): stdout is the result line
        runner.learn(args.warmup)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    kernels.timer.reset()
    kernels.timer.enabled = True
    if os.environ.get("RSLRL_BENCH_LAUNCH_EVENTS", "1") != "0":  # 0: A/B of the binding's cost
        # ~20 loss + 24 rollout-record + 1 gather launches per iteration at the default T, E x M
        kernels.timer.arm_launch_events(2 * args.steps * 50)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sys.stderr):
        runner.learn(args.steps)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed_phases = list(runner.iteration_stats_history)[-args.steps:]
    kernels.timer.enabled = False
    kernels.timer.disarm_launch_events()
    # one more iteration with the MLP GEMM launches timed (kept out of the headline timing: ~470 event
    # pairs per iteration would add host overhead to the launch-bound rollout)
    # (on one stream: the timed iteration overlaps the critic's launches with the actor's on a second stream,
    # and per-launch event spans of concurrent launches would not add up to the iteration)
    kernels.timer.mlp_enabled = True
    two = os.environ.get("RSLRL_TWO_STREAMS")
    os.environ["RSLRL_TWO_STREAMS"] = "0"
    with contextlib.redirect_stdout(sys.stderr):
        runner.learn(1)
    torch.cuda.synchronize()
    if two is None:
        os.environ.pop("RSLRL_TWO_STREAMS")
    else:
        os.environ["RSLRL_TWO_STREAMS"] = two
    kernels.timer.mlp_enabled = False
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    T, N, K = args.num_steps_per_env, args.num_envs_local, args.steps
    value = T * N * world * K / elapsed
    prof = kernels.timer.summary()
    hot = {}
    mlp = {}
    for name, s in prof.items():
        ent = {
            "launches_per_step": s["launches"] / (1 if name.startswith("linear_") else K),
            "mean_us": round(s["mean_ms"] * 1e3, 2),
            "ms_per_step": round(s["total_ms"] / (1 if name.startswith("linear_") else K), 4),
            "algorithmic_bytes_per_launch": int(s["bytes_per_launch"]),
            "achieved_GBps": round(s["bytes_per_launch"] / (s["mean_ms"] * 1e-3) / 1e9, 1),
        }
        if name in HOT_PATH:
            hot[name] = ent
        elif name.startswith("linear_"):
            ent["flops_per_launch"] = int(s["flops_per_launch"])
            ent["achieved_TFLOPs"] = round(s["flops_per_launch"] / (s["mean_ms"] * 1e-3) / 1e12, 1)
            mlp[name] = ent
    hot_ms = sum(h["ms_per_step"] for h in hot.values())
    # the timed hot-path kernels' launches (loss, rollout record, record gather) carry their own (start, stop) event
    # pair (hipExtLaunchKernel, bound inside the library): the dispatch's begin-to-end duration, what rocprofv3
    # averages; the marker span around the C-ABI call (hot_path.<kernel>.mean_us) adds the markers' dispatch latency
    # and is kept beside it.  The dominant kernel is chosen by that launch-bound kernel time per step (the marker span
    # of a 10 us kernel is ~2x its duration and would misrank it); kernels without bound events by their span.
    kernel_ms = {}
    for name, h in hot.items():
        ev_ms, ev_n = (kernels.timer.launch_events(name) if name in kernels.KernelTimer.LAUNCH_TAGS else (0.0, 0))
        if ev_n and ev_n == h["launches_per_step"] * K:
            h["launch_bound_us"] = round(ev_ms / ev_n * 1e3, 2)
            h["kernel_ms_per_step"] = round(ev_ms / K, 4)
            kernel_ms[name] = (ev_ms / K, ev_ms / ev_n, ev_n)
        else:
            kernel_ms[name] = (h["ms_per_step"], None, 0)
    dominant = max(kernel_ms, key=lambda k: kernel_ms[k][0]) if hot else None
    roofline = None
    if dominant:
        ach = hot[dominant]["achieved_GBps"]
        mean_us = hot[dominant]["mean_us"]
        timing = "HIP event span around the C-ABI call"
        _, ev_launch_ms, ev_n = kernel_ms[dominant]
        if ev_launch_ms is not None:
            mean_us = round(ev_launch_ms * 1e3, 2)
            ach = round(hot[dominant]["algorithmic_bytes_per_launch"] / (mean_us * 1e-6) / 1e9, 1)
            timing = ("HIP events bound to each launch (hipExtLaunchKernel start/stop: the dispatch's own duration, "
                      f"{ev_n} launches of the timed region); chosen as the hot-path kernel with the most launch-bound "
                      f"time per step: " + ", ".join(f"{k} {v[0] * 1e3:.1f} us" for k, v in kernel_ms.items()))
        traffic, traffic_src = pmc_traffic(PMC_NAMES.get(dominant, dominant), args.num_envs_local,
                                           args.num_steps_per_env)
        roofline = {"kernel": dominant, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "algorithmic_bytes_per_launch": hot[dominant]["algorithmic_bytes_per_launch"],
                    "mean_launch_us": mean_us, "timing": timing,
                    "call_span_us": hot[dominant]["mean_us"]}
    roofline_mlp = None
    from rsl_rl_amd.networks import fused_mlp
    mode = fused_mlp._mode
    arith_label = {fused_mlp.GEMM_H3: "h3 (REDUCED precision, opt-in): hidden-layer GEMMs on 2 fp16 planes of "
                                      "power-of-two scaled operands (22 significant bits, a1*b1 dropped); first "
                                      "and output layers x6",
                   fused_mlp.GEMM_X6: "x6: fp32 operands as 3 bf16 planes (24 significant bits), 6 bf16 MFMA "
                                      "products, fp32 accumulation (fp32-faithful; DESIGN.md s5)",
                   fused_mlp.GEMM_F32: "fp32 MFMA (exact fp32 fma chain)"}[mode]
    if mlp:
        dm = max(mlp, key=lambda k: mlp[k]["ms_per_step"])
        ach = mlp[dm]["achieved_TFLOPs"]
        if dm.endswith("/h3"):
            peak, arith = H3_PEAK_TFLOPS, "h3 split-fp16 (fp32-class, DESIGN.md s5); peak = fp16 dense / 3"
        elif mode != fused_mlp.GEMM_F32:
            peak, arith = X6_PEAK_TFLOPS, "x6 split-bf16 (fp32-class, DESIGN.md s5); peak = bf16 dense / 6"
        else:
            peak, arith = FP32_MFMA_PEAK_TFLOPS, "fp32 MFMA"
        pmc = mlp_pmc(dm)
        roofline_mlp = {"kernel": dm, "bound": "mfma", "achieved": ach, "peak": round(peak, 1), "unit": "TFLOP/s",
                        "frac": round(ach / peak, 4), "traffic": pmc["traffic_bytes"] if pmc else None,
                        "pmc": pmc,
                        "flops_per_launch": mlp[dm]["flops_per_launch"], "mean_launch_us": mlp[dm]["mean_us"],
                        "arithmetic": arith, "fp32_mfma_peak": FP32_MFMA_PEAK_TFLOPS,
                        "mlp_ms_per_step": round(sum(e["ms_per_step"] for e in mlp.values()), 3),
                        # the same launch against the HBM roofline: algorithmic bytes / event time
                        "hbm": {"achieved": mlp[dm]["achieved_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                "frac": round(mlp[dm]["achieved_GBps"] / HBM_PEAK_GBPS, 4),
                                "algorithmic_bytes_per_launch": mlp[dm]["algorithmic_bytes_per_launch"]}}

    out = {
        "metric": BASELINE_METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "gemm_arithmetic": arith_label,
        "data": "synthetic (SyntheticVecEnv: obs/reward ~ N(0,1), dones ~ Bernoulli(0.02); random-init weights)",
        "config": {
            "workload": (f"{'C3' if world == 1 and total == C3_ENVS else 'C4' if total == C4_ENVS else 'custom'}: "
                         f"{total} envs ({N} per GPU x {world}) x T={T}, obs {args.num_obs}, act {args.num_actions}, "
                         f"actor+critic MLP {args.layers}x{args.hidden} ELU, PPO E=5 M=4 adaptive-KL; "
                         f"one step = rollout + GAE + update"),
            "num_envs_per_gpu": N,
            "global_num_envs": N * world,
            "num_steps_per_env": T,
            "mini_batch_rows": N * T // 4,
            "parallelism": (f"dp{world} (env shards; one "
                            f"{'gloo (TEST: every rank on cuda:0)' if one_device else 'RCCL'} all-reduce of "
                            f"gradients + KL per mini-batch)"),
        },
        "roofline": roofline,
        "roofline_mlp": roofline_mlp,
        "mlp_kernels": mlp,
        "hot_path": hot_path_summary(hot, hot_ms, mlp, T, N),
        "phases_last_iter": {k: round(v, 4) for k, v in runner.last_iteration_stats.items() if k != "loss_dict"},
        # host-side phase times of every timed iteration (the runner's own split: collection = the rollout's host time up
        # to compute_returns, learn = update() to its statistics read-back); phases_last_iter is the extra MLP-timed one
        "phases_timed_ms": {"collection": [round(c * 1e3, 2) for c, _ in timed_phases],
                            "learn": [round(l * 1e3, 2) for _, l in timed_phases]},
        # end-to-end (value), update phase and hot path (above) reported apart
        # from the median host learn time of the timed iterations (update() to its statistics read-back; the rollout's
        # queued GPU work that drains during it is counted there too)
        "update_env_steps_per_s": round(T * N * world / statistics.median(l for _, l in timed_phases), 1),
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_extra:
        del runner, env
        torch.cuda.empty_cache()
        extra = {"C5_rnd": time_runner(args, device, rank, rnd=True)}
        extra["C5_rnd"]["workload"] = "C3 + RND (predictor/target 48->48->1 ELU, weight 1.0 x step_dt, fused record)"
        extra["C4_total_1gpu"] = time_runner(args, device, rank, num_envs=C4_ENVS)
        extra["C4_total_1gpu"]["workload"] = (f"C4's {C4_ENVS} envs on one GPU: the base point of the strong-"
                                              f"scaling curve that --gpus N partitions")
        prev = fused_mlp.set_gemm_mode(fused_mlp.GEMM_F32)
        extra["C3_fp32_mfma"] = time_runner(args, device, rank)
        extra["C3_fp32_mfma"]["workload"] = "C3 with the exact-fp32 MFMA GEMM kernels (RSLRL_GEMM_MODE=f32)"
        fused_mlp.set_gemm_mode(fused_mlp.GEMM_H3)
        extra["C3_h3_reduced_precision"] = time_runner(args, device, rank)
        extra["C3_h3_reduced_precision"]["workload"] = (
            "C3 with the hidden-layer GEMMs in h3 (RSLRL_GEMM_MODE=h3): REDUCED precision, 2 fp16 planes = 22-bit "
            "operands, a1*b1 dropped -- NOT fp32-faithful, reported for comparison only")
        fused_mlp.set_gemm_mode(prev)
        out["extra_configs"] = extra
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
