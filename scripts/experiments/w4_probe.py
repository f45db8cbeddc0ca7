"""A/B of the "w4" GEMM layout (4 waves of 128 x 64 per 128 x 256 tile, 2 waves/SIMD) against the default (8 waves
of 64 x 64) on the paired hidden forward and input gradient, one process, interleaved rounds; checks bitwise equality.

    python scripts/w4_probe.py [--rounds 5] [--iters 10]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    X6 = _lib.ARITH_X6
    for M in (98304, 393216):
        xs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev)) for _ in range(2)]
        dzs = [torch.randn(M, 256, device=dev) for _ in range(2)]
        ws = [torch.randn(256, 256, device=dev) / 16 for _ in range(2)]
        bs = [torch.randn(256, device=dev) * 0.1 for _ in range(2)]
        fimgs = [F.bimage(w, False) for w in ws]
        dimgs = [F.bimage(w, True) for w in ws]
        ops = {
            "fwd_pair": lambda: F.linear_fwd_pair(xs, bs, 256, True, fimgs, X6, [None, None], [False, False])[0],
            "dgrad_pair": lambda: F.linear_dgrad_elu_pair(dzs, xs, dimgs, X6)[0],
        }
        for name, fn in ops.items():
            res, t = {}, {"0": [], "1": []}
            for w4 in ("0", "1"):
                os.environ["RSLRL_W4"] = w4
                res[w4] = [o.clone() for o in fn()]
            same = all(torch.equal(a, b) for a, b in zip(res["0"], res["1"]))
            for _ in range(args.rounds):
                for w4 in ("0", "1"):
                    os.environ["RSLRL_W4"] = w4
                    fn()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.iters):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    t[w4].append(s.elapsed_time(e) / args.iters * 1e3)
            print(json.dumps({"op": name, "M": M, "bitwise_equal": same,
                              "default_us": round(statistics.median(t["0"]), 2),
                              "w4_us": round(statistics.median(t["1"]), 2)}), flush=True)
    os.environ["RSLRL_W4"] = "0"


if __name__ == "__main__":
    main()
