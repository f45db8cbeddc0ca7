"""Error statistics of the split-bf16 x6 GEMM vs torch fp32 (hipBLASLt), both against fp64: max, RMS and
mean signed error (a rounding bias shows up in the last), over several output widths."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rsl_rl_amd.networks.fused_mlp import bimage, linear_fwd  # noqa: E402


def stats(a, ref):
    d = a.double() - ref
    return {"max": d.abs().max().item(), "rms": d.square().mean().sqrt().item(), "mean": d.mean().item()}


res = {}
for (M, K, N, scale) in [(65536, 256, 12, True), (65536, 256, 256, True), (65536, 256, 16, False),
                         (65536, 48, 256, True), (65536, 1024, 64, True)]:
    torch.manual_seed(K + N)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / (K ** 0.5 if scale else 1.0)
    b = torch.randn(N, device="cuda")
    ref = F.linear(x.double(), w.double(), b.double())
    r = {"x6": stats(linear_fwd(x, w, b, False, bimage(w, False)), ref),
         "f32_mfma": stats(linear_fwd(x, w, b, False, None), ref),
         "torch_fp32": stats(F.linear(x, w, b), ref),
         "ref_rms": ref.square().mean().sqrt().item()}
    res[f"{M}x{K}x{N}{'' if scale else '_unscaled'}"] = r
print(json.dumps(res, indent=1))
