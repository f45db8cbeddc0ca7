"""Probe: the x6 fused linear kernels at C3 mini-batch shapes (M = 393216), each timed with and without the
unrolled look-ahead main loop (RSLRL_H3_DEEP bit mask, read per call) in one process.  The look-ahead depth
is compile-time (RSLRL_X6_DEPTH): run once per library build (RSLRL_AMD_LIB selects the .so)."""

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    dev = torch.device("cuda:0")
    M = int(os.environ.get("PROBE_M", 393216))
    torch.manual_seed(0)
    x = F.elu(torch.randn(M, 256, device=dev))
    dz = torch.randn(M, 256, device=dev) * 1e-6
    w = torch.randn(256, 256, device=dev) / 16
    b = torch.randn(256, device=dev) * 0.1
    wo = torch.randn(12, 256, device=dev) / 16
    bo = torch.randn(12, device=dev)
    wv = torch.randn(1, 256, device=dev) / 16
    bv = torch.randn(1, device=dev)
    X6 = _lib.ARITH_X6
    oimg, vimg = fused_mlp.bimages([(wo, False, _lib.BIMAGE_LAYOUT_OUT), (wv, False, _lib.BIMAGE_LAYOUT_OUT)])
    im6f, im6t = fused_mlp.bimages([(w, False), (w, True)])
    ax, adz = x.abs().amax().reshape(1), dz.abs().amax().reshape(1)
    cases = {
        "fwd": lambda: fused_mlp.linear_fwd_ex(x, b, 256, True, im6f, X6, ax, True),
        "fwd_out12": lambda: fused_mlp.linear_fwd_out_ex(x, b, 256, im6f, X6, ax, bo, oimg, True),
        "fwd_out1": lambda: fused_mlp.linear_fwd_out_ex(x, b, 256, im6f, X6, ax, bv, vimg, True),
        "dgrad": lambda: fused_mlp.linear_dgrad_elu_ex(dz, x, im6t, X6, adz, True),
        "fwd_noamax": lambda: fused_mlp.linear_fwd_ex(x, b, 256, True, im6f, X6, ax, False),
        "fwd16": lambda: fused_mlp.linear_fwd_ex(x, b, 256, True, im6f, X6, ax, False),
        "fwd16_minw2": lambda: fused_mlp.linear_fwd_ex(x, b, 256, True, im6f, X6, ax, False),
    }
    knobs = {"fwd16": {"RSLRL_X6_SHAPE": "16"}, "fwd16_minw2": {"RSLRL_X6_SHAPE": "16", "RSLRL_X6S_MINW": "2"}}
    res = {"lib": os.environ.get("RSLRL_AMD_LIB", "default")}
    for name, fn in cases.items():
        for k, v in knobs.get(name, {}).items():
            os.environ[k] = v
        r = {}
        masks = ((0xff, "deep"),) if os.environ.get("PROBE_DEEP_ONLY") else ((0, "loop1"), (0xff, "deep"))
        for mask, tag in masks:
            os.environ["RSLRL_H3_DEEP"] = str(mask)
            r[tag] = t(fn)
        os.environ.pop("RSLRL_H3_DEEP")
        for k in knobs.get(name, {}):
            os.environ.pop(k)
        res[name] = r
    res["wgrad"] = t(lambda: fused_mlp.linear_wgrad(dz, x, X6, adz, ax))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
