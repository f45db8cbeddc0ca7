"""Outputs of the paired hidden forward / input gradient on fixed random inputs, saved for a bitwise comparison of two
library builds (RSLRL_AMD_LIB): python scripts/gemm_dump.py OUT.pt [--M 393216]; python scripts/gemm_dump.py --cmp A B"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--M", type=int, default=98304)
    ap.add_argument("--cmp", nargs=2)
    args = ap.parse_args()
    if args.cmp:
        a, b = (torch.load(f, weights_only=True) for f in args.cmp)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print({"compared": sorted(a), "differ": bad})
        for k in bad:
            d = (a[k] - b[k]).abs()
            nz = (a[k] != b[k]).nonzero()
            print(k, {"max_abs": d.max().item(), "max_ref": b[k].abs().max().item(), "n_differ": nz.shape[0],
                      "of": a[k].numel(), "first": nz[:8].tolist(),
                      "rows_mod_32": torch.bincount(nz[:, 0] % 32, minlength=32).tolist(),
                      "cols_mod_32": torch.bincount(nz[:, 1] % 32, minlength=32).tolist(),
                      "nan_a": torch.isnan(a[k]).sum().item(), "nan_b": torch.isnan(b[k]).sum().item()})
        sys.exit(1 if bad else 0)
    from rsl_rl_amd import _lib
    from rsl_rl_amd.networks import fused_mlp as F

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    M, X6 = args.M, _lib.ARITH_X6
    xs = [torch.nn.functional.elu(torch.randn(M, 256, device=dev, generator=g)) for _ in range(2)]
    dzs = [torch.randn(M, 256, device=dev, generator=g) for _ in range(2)]
    ws = [torch.randn(256, 256, device=dev, generator=g) / 16 for _ in range(2)]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(2)]
    fimgs = [F.bimage(w, False) for w in ws]
    dimgs = [F.bimage(w, True) for w in ws]
    out = {}
    rep = {}
    for w4 in ("0", "1"):  # run-to-run determinism inside the process first
        os.environ["RSLRL_W4"] = w4
        runs = [[t.clone() for t in F.linear_fwd_pair(xs, bs, 256, True, fimgs, X6, [None, None], [False, False])[0]]
                + [t.clone() for t in F.linear_dgrad_elu_pair(dzs, xs, dimgs, X6)[0]] for _ in range(4)]
        rep[w4] = [all(torch.equal(a, b) for a, b in zip(runs[0], r)) for r in runs[1:]]
    print({"deterministic_in_process": rep}, flush=True)
    for w4 in ("0", "1"):
        os.environ["RSLRL_W4"] = w4
        f = F.linear_fwd_pair(xs, bs, 256, True, fimgs, X6, [None, None], [False, False])[0]
        d = F.linear_dgrad_elu_pair(dzs, xs, dimgs, X6)[0]
        for i in range(2):
            out[f"fwd{i}_w4{w4}"] = f[i].cpu()
            out[f"dgrad{i}_w4{w4}"] = d[i].cpu()
        out[f"fwd_single_w4{w4}"] = F.linear_fwd_ex(xs[0], bs[0], 256, True, fimgs[0], X6)[0].cpu()
    torch.save(out, args.out)


if __name__ == "__main__":
    main()
