"""The update's 256x256 x6 GEMM pairs at C3's mini-batch (393,216 rows), each launched --iters times on random data,
for rocprofv3 kernel-trace / PMC passes (scripts/mlp_pmc.sh): the hidden forward pair (bias + ELU), the hidden
input-gradient pair (dZ W * ELU'(H), the w4 kernel) and the weight-gradient pair (dZ^T H + column sums, folds
deferred as in the update).

    python scripts/mlp_pair_probe.py [--iters 10] [--ops fwd,dgrad,wgrad]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--M", type=int, default=393216)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    X6 = _lib.ARITH_X6
    M = args.M
    xs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev)) for _ in range(2)]
    dzs = [torch.randn(M, 256, device=dev) * 1e-3 for _ in range(2)]
    ws = [torch.randn(256, 256, device=dev) / 16 for _ in range(2)]
    bs = [torch.randn(256, device=dev) * 0.1 for _ in range(2)]
    fimgs = [F.bimage(w, False) for w in ws]
    dimgs = [F.bimage(w, True) for w in ws]
    ops = {
        "fwd": lambda: F.linear_fwd_pair(xs, bs, 256, True, fimgs, X6, [None, None], [False, False]),
        "dgrad": lambda: F.linear_dgrad_elu_pair(dzs, xs, dimgs, X6),
        "wgrad": lambda: F.linear_wgrad_pair(dzs, xs, X6, bias_side=1),
    }
    out = {}
    for name in args.ops.split(","):
        fn = ops[name]
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(s.elapsed_time(e) / args.iters * 1e3, 1)
    print(json.dumps({"M": M, **out}), flush=True)


if __name__ == "__main__":
    main()
