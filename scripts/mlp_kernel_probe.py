"""Probe: fused MFMA linear kernels (csrc/mlp_gemm.hip) vs torch (hipBLASLt GEMM + ATen ELU) at C3
mini-batch shapes (M = 393216)."""

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd.networks.fused_mlp import linear_dgrad_elu, linear_fwd  # noqa: E402


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
    M = 393216
    res = {}
    for K, N in ((256, 256), (48, 256)):
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        fl = 2.0 * M * K * N
        ours = t(lambda: linear_fwd(x, w, b, True))
        ref = t(lambda: F.elu(F.linear(x, w, b)))
        gemm = t(lambda: F.linear(x, w, b))
        res[f"fwd_elu_{K}x{N}"] = {"fused_us": ours, "torch_gemm_elu_us": ref, "torch_gemm_only_us": gemm,
                                   "fused_TFLOPs": fl / ours / 1e6, "torch_gemm_TFLOPs": fl / gemm / 1e6}
    for N, K in ((256, 256), (12, 256)):
        dz = torch.randn(M, N, device=dev)
        w = torch.randn(N, K, device=dev)
        h = F.elu(torch.randn(M, K, device=dev))
        fl = 2.0 * M * K * N
        ours = t(lambda: linear_dgrad_elu(dz, w, h))

        def ref_fn():
            d = dz.mm(w)
            d = torch.where(h > 0, d, d * (h + 1))
            return d, d.sum(0)

        ref = t(ref_fn)
        res[f"dgrad_elu_{N}to{K}"] = {"fused_us": ours, "torch_us": ref, "fused_TFLOPs": fl / ours / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
