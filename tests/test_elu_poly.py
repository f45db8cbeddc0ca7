"""The ELU's negative branch on the GPU GEMM epilogues (mlp_gemm.hip elu_neg, mlp_fwd_stream.hip fs_elu_neg,
rollout_mlp.hip rm_elu_neg): a degree-5
polynomial for expm1 on [-0.5, 0], exp(v) - 1 below.  Host check of the polynomial part, evaluated as the kernels do
(fp32 Horner with fused multiply-adds, then one fp32 multiply), against expm1 in fp64: within 1.3 ulp of fp32 on
every 97th fp32 in [-0.5, 0); and every kernel carries the same coefficients (their outputs are compared bit for bit by
the GPU tests)."""

import os
import re

import numpy as np

from conftest import ROOT

SRC = os.path.join(ROOT, "rsl_rl_amd", "csrc")


def coefficients(path, fn):
    text = open(os.path.join(SRC, path)).read()
    body = text[text.index(f"float {fn}(float v)"):]
    body = body[:body.index("const float poly")]
    lits = [np.float32(x) for x in re.findall(r"([-+]?\d*\.\d+(?:e[-+]?\d+)?)f", body)]
    # __fmaf_rn(v, c_top, c_next) then __fmaf_rn(v, t, c): the literals in source order, highest degree first
    return lits


def horner(c, v):
    v64 = v.astype(np.float64)
    t = np.full_like(v, c[0])
    for k in c[1:]:
        t = (v64 * t.astype(np.float64) + np.float64(k)).astype(np.float32)  # fp32 product exact in fp64: one rounding
    return (v * t).astype(np.float32)


def test_elu_polynomial_is_fp32_faithful():
    c = coefficients("mlp_gemm.hip", "elu_neg")
    assert len(c) == 6, c
    bits = np.arange(0x80000001, 0xBF000000, 97, dtype=np.uint64).astype(np.uint32)
    v = bits.view(np.float32)
    ref = np.expm1(v.astype(np.float64))
    ulp = np.abs(horner(c, v).astype(np.float64) - ref) / np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    assert ulp.max() <= 1.3, ulp.max()


def test_every_epilogue_uses_the_same_polynomial():
    c = coefficients("mlp_gemm.hip", "elu_neg")
    assert c == coefficients("mlp_fwd_stream.hip", "fs_elu_neg")
    assert c == coefficients("rollout_mlp.hip", "rm_elu_neg")
