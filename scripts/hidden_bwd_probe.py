"""Time the fused hidden-layer backward (rslrl_hidden_bwd_pair) against the launches it replaces (the weight-gradient
pair with bias sums + the input-gradient pair) at C3's 393,216-row mini-batch and the 16384-env share's 98,304 rows,
alternating the two forms in one process; HIP events on the current stream.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402


def problem(M, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dz = torch.randn(M, 256, device="cuda", generator=g) * 0.01
    h = torch.nn.functional.elu(torch.randn(M, 256, device="cuda", generator=g))
    w = torch.randn(256, 256, device="cuda", generator=g) / 16
    return dz, h, w


def timed(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) * 1e3 for a, b in ev)


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["fused", "separate"], help="launch only this form --iters times (profiling)")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--M", type=int, default=0)
    ap.add_argument("--variants", default="", help="comma-separated RSLRL_HB_VARIANT values 'BD:LA' timed in turn")
    args = ap.parse_args()
    out = {}
    rounds = int(os.environ.get("PROBE_ROUNDS", "3"))
    for M in ((args.M,) if args.M else (393216, 98304)):
        p = [problem(M, 1), problem(M, 2)]
        dzs, hs = [q[0] for q in p], [q[1] for q in p]
        imgs = fused_mlp.bimages([(q[2], True) for q in p])

        def fused():
            folds = fused_mlp._FoldBatch()
            fused_mlp.hidden_bwd_pair(dzs, hs, imgs, defer=folds)
            folds.run(dzs[0].device)

        def separate():
            folds = fused_mlp._FoldBatch()
            fused_mlp.linear_wgrad_pair(dzs, hs, bias_side=1, defer=folds)
            fused_mlp.linear_dgrad_elu_pair(dzs, hs, imgs, _lib.ARITH_X6)
            folds.run(dzs[0].device)

        def kern_fused():
            fused_mlp.hidden_bwd_pair(dzs, hs, imgs, defer=fused_mlp._FoldBatch())

        for f in (fused, separate):
            f()
        torch.cuda.synchronize()
        if args.only:
            f = fused if args.only == "fused" else separate
            for _ in range(args.iters):
                f()
            torch.cuda.synchronize()
            continue
        res = {"fused": [], "separate": [], "fused_kernel_only": []}
        variants = [v.replace(":", ",") for v in args.variants.split(",") if v]
        for v in variants:
            res["variant " + v] = []
        for _ in range(rounds):
            res["fused"] += timed(fused, 10)
            res["separate"] += timed(separate, 10)
            res["fused_kernel_only"] += timed(kern_fused, 10)
            for v in variants:
                os.environ["RSLRL_HB_VARIANT"] = v
                res["variant " + v] += timed(kern_fused, 10)
                os.environ.pop("RSLRL_HB_VARIANT")
        out[M] = {k: {"median_us": round(sorted(v)[len(v) // 2], 1), "min_us": round(min(v), 1)} for k, v in res.items()}
        del p, dzs, hs, imgs
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
