"""Standalone timing of the hot-path kernels at config C3 shapes (N=65536, T=24, O=48, A=12, M=4).

Times each C-ABI entry point with HIP events over many launches on the current stream, rotating over
enough input sets that the working set exceeds the 256 MB Infinity Cache, and prints algorithmic GB/s.
Used to iterate on kernels; bench.py reports the same quantities live inside the real training step.

    python scripts/hotpath_microbench.py [--iters 50] [--only loss,gather,gae]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import kernels  # noqa: E402


def timeit(fn, iters):
    fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="gae,normalize,gather,loss,loss_perrow")
    args = ap.parse_args()
    only = set(args.only.split(","))
    dev = torch.device("cuda:0")
    T, N, O, A, M = 24, int(os.environ.get("MICROBENCH_ENVS", "65536")), 48, 12, 4
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}

    if "gae" in only or "normalize" in only:
        sets = []
        for _ in range(12):  # 12 x 27 MB > 256 MB
            v = torch.randn(T, N, 1, device=dev, generator=g)
            r = torch.randn(T, N, 1, device=dev, generator=g)
            d = (torch.rand(T, N, 1, device=dev, generator=g) < 0.02).to(torch.uint8)
            lv = torch.randn(N, 1, device=dev, generator=g)
            sets.append((v, r, d, lv, torch.empty_like(v), torch.empty_like(v)))
        if "gae" in only:
            us = timeit(lambda i: kernels.compute_returns(*sets[i % 12][:4], 0.99, 0.95, False, *sets[i % 12][4:]),
                        args.iters)
            res["gae_scan"] = {"us": us, "GBps": (17 * T * N + 4 * N) / us / 1e3}
            us2 = timeit(lambda i: kernels.compute_returns(*sets[i % 12][:4], 0.99, 0.95, True, *sets[i % 12][4:]),
                         args.iters)
            res["compute_returns_normalized"] = {"us": us2, "GBps": (25 * T * N + 4 * N) / us2 / 1e3}
        if "normalize" in only:
            us = timeit(lambda i: kernels.normalize_advantages_(sets[i % 12][5].view(-1)), args.iters)
            res["normalize_standalone"] = {"us": us, "GBps": 12 * T * N / us / 1e3}

    if "gather" in only:
        rows = T * N
        srcs = {"obs": torch.randn(rows, O, device=dev, generator=g)}
        for k in ("actions", "mu", "sigma"):
            srcs[k] = torch.randn(rows, A, device=dev, generator=g)
        for k in ("values", "returns", "logp", "adv"):
            srcs[k] = torch.randn(rows, 1, device=dev, generator=g)
        dsts = {k: torch.empty_like(v) for k, v in srcs.items()}
        idx = torch.randperm(rows, device=dev, generator=g).to(torch.int32)
        pairs = [(srcs[k], dsts[k]) for k in srcs]
        moved = sum(2 * v.numel() * 4 for v in srcs.values()) + 4 * rows
        us = timeit(lambda i: kernels.gather_rows(pairs, idx), max(5, args.iters // 5))
        res["gather_rows"] = {"us": us, "GBps": moved / us / 1e3, "bytes": moved}

    for mode in ("loss", "loss_perrow"):
        if mode not in only:
            continue
        B = N * T // M
        sets = []
        for _ in range(4):  # 4 mini-batches x ~110 MB
            mu = torch.randn(B, A, device=dev, generator=g)
            sig = (0.5 + torch.rand(A if mode == "loss" else (B, A), device=dev, generator=g)).contiguous()
            x = torch.randn(B, A, device=dev, generator=g)
            omu = torch.randn(B, A, device=dev, generator=g)
            # as a rollout stores it: one old sigma per action for every sample with a shared std (the training
            # step's case), per row otherwise
            osig = ((0.5 + torch.rand(A, device=dev, generator=g)).expand(B, A).contiguous() if mode == "loss"
                    else 0.5 + torch.rand(B, A, device=dev, generator=g))
            sc = [torch.randn(B, 1, device=dev, generator=g) for _ in range(5)]
            sets.append((mu, sig, sc[0], x, sc[1], sc[2], sc[3], sc[4], omu, osig))
        outs = [(torch.empty(B, A, device=dev), torch.empty(sets[0][1].shape, device=dev),
                 torch.empty(B, 1, device=dev), torch.empty(8, device=dev)) for _ in range(4)]

        def run(i):
            o = outs[i % 4]
            kernels.ppo_loss_fwd_bwd(*sets[i % 4], grad_mu=o[0], grad_sigma=o[1], grad_values=o[2], stats=o[3])

        us = timeit(run, args.iters)
        per_row = 4 * (4 * A + 5) + 4 * (A + 1) + (8 * A if mode == "loss_perrow" else 0)
        res[mode] = {"us": us, "GBps": per_row * B / us / 1e3, "bytes": per_row * B}

    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
