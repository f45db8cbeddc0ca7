"""Probe: fused MFMA linear kernels (csrc/mlp_gemm.hip) in both arithmetic modes (f32 MFMA, split-bf16
x6) vs torch (hipBLASLt GEMM + ATen ELU) at C3 mini-batch shapes (M = 393216): time, TFLOP/s and the
max error of each against an fp64 evaluation of the same layer."""

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd.networks.fused_mlp import bimage, linear_dgrad_elu, linear_fwd, linear_wgrad  # noqa: E402
from rsl_rl_amd.networks.linear import _splitk_weight_grad  # noqa: E402

MODES = {"f32": False, "x6": True}


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


def rel_err(a, ref):
    return ((a.double() - ref).abs().max() / ref.abs().max()).item()


def main():
    dev = "cuda"
    M = int(os.environ.get("PROBE_M", 393216))
    res = {}
    only = os.environ.get("PROBE_ONLY")  # "fwd" | "dgrad": one direction (profiling runs)
    fwd_shapes = () if only == "dgrad" else ((256, 256),) if only == "fwd" else ((256, 256), (48, 256))
    dgrad_shapes = () if only == "fwd" else ((256, 256),) if only == "dgrad" else ((256, 256), (12, 256))
    modes = {k: v for k, v in MODES.items() if not only or k == "x6"}
    for K, N in fwd_shapes:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        fl = 2.0 * M * K * N
        ref64 = F.elu(F.linear(x.double(), w.double(), b.double()))
        r = {}
        for name, x6 in modes.items():
            img = bimage(w, False) if x6 else None
            us = t(lambda: linear_fwd(x, w, b, True, img))
            r[name] = {"us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1),
                       "rel_err": rel_err(linear_fwd(x, w, b, True, img), ref64)}
            if x6:
                r[name]["bimage_us"] = round(t(lambda: bimage(w, False)), 1)
        gemm = t(lambda: F.linear(x, w, b))
        r["torch"] = {"gemm_us": round(gemm, 1), "gemm_elu_us": round(t(lambda: F.elu(F.linear(x, w, b))), 1),
                      "TFLOPs": round(fl / gemm / 1e6, 1), "rel_err": rel_err(F.elu(F.linear(x, w, b)), ref64)}
        res[f"fwd_elu_{K}x{N}"] = r
        del ref64
    for N, K in dgrad_shapes:
        dz = torch.randn(M, N, device=dev)
        w = torch.randn(N, K, device=dev)
        h = F.elu(torch.randn(M, K, device=dev))
        fl = 2.0 * M * K * N
        d64 = dz.double().mm(w.double())
        ref64 = torch.where(h > 0, d64, d64 * (h.double() + 1))
        del d64
        r = {}
        for name, x6 in modes.items():
            img = bimage(w, True) if x6 else None
            us = t(lambda: linear_dgrad_elu(dz, w, h, img))
            r[name] = {"us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1),
                       "rel_err": rel_err(linear_dgrad_elu(dz, w, h, img)[0], ref64)}

        def ref_fn():
            d = dz.mm(w)
            d = torch.where(h > 0, d, d * (h + 1))
            return d, d.sum(0)

        r["torch"] = {"us": round(t(ref_fn), 1), "rel_err": rel_err(ref_fn()[0], ref64)}
        res[f"dgrad_elu_{N}to{K}"] = r
        del ref64
    wgrad_shapes = () if only in ("fwd", "dgrad") else ((256, 256), (256, 48), (12, 256))
    for N, K in wgrad_shapes:
        dz = torch.randn(M, N, device=dev)
        x = torch.randn(M, K, device=dev)
        fl = 2.0 * M * K * N
        ref64 = dz.double().t().mm(x.double())
        us = t(lambda: linear_wgrad(dz, x))
        tsk = t(lambda: _splitk_weight_grad(dz, x))
        res[f"wgrad_{N}x{K}"] = {
            "x6": {"us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1), "rel_err": rel_err(linear_wgrad(dz, x), ref64)},
            "torch_splitk": {"us": round(tsk, 1), "TFLOPs": round(fl / tsk / 1e6, 1),
                             "rel_err": rel_err(_splitk_weight_grad(dz, x), ref64)}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
