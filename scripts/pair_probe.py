"""Actor + critic hidden-layer input gradients: two launches vs one pair launch (rslrl_linear_gemm_pair), x6, at
the update's mini-batch rows for 65536 / 32768 / 16384 envs per GPU.  Interleaved rounds in one process; checks the
pair is bit-identical to the singles.

    python scripts/pair_probe.py [--rounds 5] [--iters 20]
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
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    res = {}
    for M in (98304, 196608, 393216):
        dzs = [torch.randn(M, 256, device=dev) for _ in range(2)]
        hs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev)) for _ in range(2)]
        ws = [torch.randn(256, 256, device=dev) / 16 for _ in range(2)]
        imgs = [F.bimage(w, True) for w in ws]
        X6 = _lib.ARITH_X6

        def singles():
            return [F.linear_dgrad_elu_ex(dzs[i], hs[i], imgs[i], X6, want_db=False)[0] for i in range(2)]

        def pair():
            return F.linear_dgrad_elu_pair(dzs, hs, imgs, X6)[0]

        a, b = singles(), pair()
        torch.cuda.synchronize()
        same = all(torch.equal(x, y) for x, y in zip(a, b))
        t = {"singles": [], "pair": []}
        for _ in range(args.rounds):
            for name, fn in (("singles", singles), ("pair", pair)):
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                t[name].append(s.elapsed_time(e) / args.iters * 1e3)
        res[M] = {"bitwise_equal": same, **{k: round(statistics.median(v), 2) for k, v in t.items()},
                  "min": {k: round(min(v), 2) for k, v in t.items()}}
        print(json.dumps({"dgrad": M, **res[M]}), flush=True)

        # weight gradients: hidden 256x256 (+ bias of dz) and the first layer's (x^T dz)^T form (48 x 256, bias of dz)
        x48 = [torch.randn(M, 48, device=dev) for _ in range(2)]
        for name, A_, B_, side in (("wgrad256", dzs, hs, 1), ("wgrad48", x48, dzs, 2)):
            def w_singles():
                return [F.linear_wgrad(A_[i], B_[i], bias_side=side) for i in range(2)]

            def w_pair():
                return F.linear_wgrad_pair(A_, B_, bias_side=side)

            a, b = w_singles(), w_pair()
            ref = [A_[i].double().t().mm(B_[i].double()) for i in range(2)]
            err = lambda d, r: ((d.double() - r).abs().max() / r.abs().max()).item()  # noqa: E731
            errs = {"single": max(err(a[i][0], ref[i]) for i in range(2)),
                    "pair": max(err(b[i][0], ref[i]) for i in range(2))}
            t = {"singles": [], "pair": []}
            for _ in range(args.rounds):
                for nm, fn in (("singles", w_singles), ("pair", w_pair)):
                    fn()
                    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s_.record()
                    for _ in range(args.iters):
                        fn()
                    e_.record()
                    torch.cuda.synchronize()
                    t[nm].append(s_.elapsed_time(e_) / args.iters * 1e3)
            print(json.dumps({name: M, "max_rel_err_vs_fp64": errs,
                              **{k: round(statistics.median(v), 2) for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
