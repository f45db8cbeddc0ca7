"""In-process A/B of the x6 GEMM tile layouts on the update's paired hidden forward and input gradient (interleaved
rounds, one process, random data; outputs checked bitwise against the default layout).  A variant is a set of
environment knobs read per launch by the library (RSLRL_W4, RSLRL_W8).

    python scripts/gemm_ab.py [--rounds 5] [--iters 10] [--M 393216,98304] [--variants base,w4,w8]
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

VARIANTS = {
    "base": {"RSLRL_W4": "0", "RSLRL_W8": "0"},
    "w4": {"RSLRL_W4": "1", "RSLRL_W8": "0"},
    "w8": {"RSLRL_W4": "0", "RSLRL_W8": "1"},
    "default": {"RSLRL_W4": None, "RSLRL_W8": None},
}


def setenv(v):
    for k, x in VARIANTS[v].items():
        if x is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--M", default="393216,98304")
    ap.add_argument("--variants", default="base,w4,w8")
    ap.add_argument("--ops", default="fwd,dgrad")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    X6 = _lib.ARITH_X6
    variants = args.variants.split(",")
    for M in [int(m) for m in args.M.split(",")]:
        xs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev)) for _ in range(2)]
        dzs = [torch.randn(M, 256, device=dev) * 1e-3 for _ in range(2)]
        ws = [torch.randn(256, 256, device=dev) / 16 for _ in range(2)]
        bs = [torch.randn(256, device=dev) * 0.1 for _ in range(2)]
        fimgs = [F.bimage(w, False) for w in ws]
        dimgs = [F.bimage(w, True) for w in ws]
        ops = {
            "fwd": lambda: F.linear_fwd_pair(xs, bs, 256, True, fimgs, X6, [None, None], [False, False])[0],
            "dgrad": lambda: F.linear_dgrad_elu_pair(dzs, xs, dimgs, X6)[0],
        }
        for name in args.ops.split(","):
            fn = ops[name]
            res, t = {}, {v: [] for v in variants}
            for v in variants:
                setenv(v)
                res[v] = [o.clone() for o in fn()]
            same = {v: all(torch.equal(a, b) for a, b in zip(res[variants[0]], res[v])) for v in variants}
            for _ in range(args.rounds):
                for v in variants:
                    setenv(v)
                    fn()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.iters):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    t[v].append(s.elapsed_time(e) / args.iters * 1e3)
            print(json.dumps({"op": name, "M": M, "bitwise_equal_to_" + variants[0]: same,
                              "median_us": {v: round(statistics.median(t[v]), 1) for v in variants},
                              "min_us": {v: round(min(t[v]), 1) for v in variants}}), flush=True)
    setenv("default")


if __name__ == "__main__":
    main()
