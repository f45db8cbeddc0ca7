"""Loss kernel in the bench's context: each launch preceded by an MFMA-heavy GEMM (as in the update, where the
actor/critic output layers run right before it) vs back to back.  Reports the per-launch HIP-event span (the
bench's measure) for both; run under rocprofv3 --kernel-trace --stats for the kernel durations.

    python scripts/loss_incontext.py [--iters 200] [--heat none|bf16|fp32]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--heat", default="bf16")
    ap.add_argument("--gv-pad", action="store_true", help="d V into column 0 of a [B, 4] buffer (the update's layout)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    T, N, A, M = 24, int(os.environ.get("MICROBENCH_ENVS", "65536")), 12, 4
    B = N * T // M
    g = torch.Generator(device=dev).manual_seed(0)
    sets = []
    for _ in range(4):
        mu = torch.randn(B, A, device=dev, generator=g)
        sig = (0.5 + torch.rand(A, device=dev, generator=g)).contiguous()
        x = torch.randn(B, A, device=dev, generator=g)
        omu = torch.randn(B, A, device=dev, generator=g)
        osig = (0.5 + torch.rand(A, device=dev, generator=g)).expand(B, A).contiguous()
        sc = [torch.randn(B, 1, device=dev, generator=g) for _ in range(5)]
        sets.append((mu, sig, sc[0], x, sc[1], sc[2], sc[3], sc[4], omu, osig))
    outs = [(torch.empty(B, A, device=dev), torch.empty(A, device=dev),
             torch.zeros(B, 4, device=dev)[:, :1] if args.gv_pad else torch.empty(B, 1, device=dev),
             torch.empty(8, device=dev)) for _ in range(4)]
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}.get(args.heat)
    if dt is not None:
        ha = torch.randn(8192, 4096, device=dev, generator=g).to(dt)
        hb = torch.randn(4096, 4096, device=dev, generator=g).to(dt)
        hc = torch.empty(8192, 4096, device=dev, dtype=dt)

    def heat():
        if dt is not None:
            torch.mm(ha, hb, out=hc)

    def loss(i):
        o = outs[i % 4]
        kernels.ppo_loss_fwd_bwd(*sets[i % 4], grad_mu=o[0], grad_sigma=o[1], grad_values=o[2], stats=o[3])

    for i in range(20):
        heat()
        loss(i)
    torch.cuda.synchronize()
    kernels.timer.reset()
    kernels.timer.enabled = True
    for i in range(args.iters):
        heat()
        loss(i)
    torch.cuda.synchronize()
    kernels.timer.enabled = False
    s = kernels.timer.summary()["ppo_loss"]
    print(json.dumps({"heat": args.heat, "gv_pad": args.gv_pad, "envs": N, "span_us": s["mean_ms"] * 1e3,
                      "frac": s["bytes_per_launch"] / (s["mean_ms"] * 1e-3) / 8e12}))


if __name__ == "__main__":
    main()
