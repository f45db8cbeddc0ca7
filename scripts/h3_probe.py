"""Probe: the h3 fused linear kernels at C3 mini-batch shapes (M = 393216), each timed with and without the
unrolled look-ahead main loop (RSLRL_H3_DEEP bit mask, read per call) in one process, plus the x6 kernels of
the same shapes -- the box-to-box clock spread makes cross-run comparisons of a few per cent meaningless."""

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
    H3, X6 = _lib.ARITH_H3, _lib.ARITH_X6
    im3f, im3t, oimg = fused_mlp.bimages([(w, False, _lib.BIMAGE_LAYOUT_H3), (w, True, _lib.BIMAGE_LAYOUT_H3),
                                          (wo, False, _lib.BIMAGE_LAYOUT_OUT)])
    im6f, im6t = fused_mlp.bimages([(w, False), (w, True)])
    ax, adz = x.abs().amax().reshape(1), dz.abs().amax().reshape(1)
    cases = {
        "fwd": (lambda a: fused_mlp.linear_fwd_ex(x, b, 256, True, im3f if a == H3 else im6f, a, ax, True)),
        "fwd_out12": (lambda a: fused_mlp.linear_fwd_out_ex(x, b, 256, im3f if a == H3 else im6f, a, ax, bo, oimg,
                                                            True)),
        "dgrad": (lambda a: fused_mlp.linear_dgrad_elu_ex(dz, x, im3t if a == H3 else im6t, a, adz, True)),
        "wgrad": (lambda a: fused_mlp.linear_wgrad(dz, x, a, adz, ax)),
    }
    res = {}
    for name, fn in cases.items():
        r = {"x6": t(lambda: fn(X6))}
        for mask, tag in ((0, "h3"), (0xff, "h3_deep")):
            os.environ["RSLRL_H3_DEEP"] = str(mask)
            r[tag] = t(lambda: fn(H3))
        os.environ.pop("RSLRL_H3_DEEP")
        r["h3_default"] = t(lambda: fn(H3))
        res[name] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
