"""Probe: weight-gradient GEMM dW = dY^T X over a huge batch (K = 393216 rows) -- hipBLASLt direct vs
split-K batched GEMM + reduction.  Used to pick the MLP backward strategy (MLP section)."""

import json

import torch


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = "cuda"
    B = 393216
    res = {}
    for out_f, in_f in ((256, 256), (256, 48), (12, 256), (1, 256)):
        X = torch.randn(B, in_f, device=dev)
        dY = torch.randn(B, out_f, device=dev)
        flop = 2.0 * B * in_f * out_f
        r = {"direct_us": t(lambda: dY.t().mm(X))}
        ref = dY.t().mm(X)
        for S in (4, 8, 16, 32, 64, 128):
            Xs = X.view(S, B // S, in_f)
            dYs = dY.view(S, B // S, out_f)

            def f():
                return torch.bmm(dYs.transpose(1, 2), Xs).sum(0)

            r[f"splitk{S}_us"] = t(f)
            err = (f() - ref).abs().max().item() / ref.abs().max().item()
            r[f"splitk{S}_relerr"] = err
        best = min(v for k, v in r.items() if k.endswith("_us"))
        r["best_TFLOPs"] = flop / best / 1e6
        r["direct_TFLOPs"] = flop / r["direct_us"] / 1e6
        res[f"{out_f}x{in_f}"] = r
    # forward-like GEMM for reference
    X = torch.randn(B, 256, device=dev)
    W = torch.randn(256, 256, device=dev)
    us = t(lambda: torch.nn.functional.linear(X, W))
    res["fwd_256x256_us"] = us
    res["fwd_256x256_TFLOPs"] = 2.0 * B * 256 * 256 / us / 1e6
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
