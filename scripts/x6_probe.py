"""Probe: the x6 fused linear kernels at C3 mini-batch shapes (M = 393216, as the x6 training path calls them: no
amax), each timed under several per-call knobs in one process (the box-to-box clock spread makes cross-run
comparisons of a few per cent meaningless).  PROBE_VARIANTS: JSON {tag: {ENV: value}}; default compares the
look-ahead loop with B staged through LDS against B fragments loaded from global memory (RSLRL_X6_DIRECTB)."""

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
    x48 = torch.randn(M, 48, device=dev)
    dz = torch.randn(M, 256, device=dev) * 1e-6
    w = torch.randn(256, 256, device=dev) / 16
    w48 = torch.randn(256, 48, device=dev) / 7
    b = torch.randn(256, device=dev) * 0.1
    wo = torch.randn(12, 256, device=dev) / 16
    bo = torch.randn(12, device=dev)
    wv = torch.randn(1, 256, device=dev) / 16
    bv = torch.randn(1, device=dev)
    X6 = _lib.ARITH_X6
    oimg, vimg = fused_mlp.bimages([(wo, False, _lib.BIMAGE_LAYOUT_OUT), (wv, False, _lib.BIMAGE_LAYOUT_OUT)])
    im6f, im6t, im48 = fused_mlp.bimages([(w, False), (w, True), (w48, False)])
    cases = {
        "fwd48": lambda: fused_mlp.linear_fwd_ex(x48, b, 256, True, im48, X6, None, False),
        "fwd": lambda: fused_mlp.linear_fwd_ex(x, b, 256, True, im6f, X6, None, False),
        "fwd_out12": lambda: fused_mlp.linear_fwd_out_ex(x, b, 256, im6f, X6, None, bo, oimg, True),
        "fwd_out1": lambda: fused_mlp.linear_fwd_out_ex(x, b, 256, im6f, X6, None, bv, vimg, True),
        "dgrad": lambda: fused_mlp.linear_dgrad_elu_ex(dz, x, im6t, X6, None, False),
        "wgrad": lambda: fused_mlp.linear_wgrad(dz, x, X6),
        "wgrad48": lambda: fused_mlp.linear_wgrad(x48, dz, X6),
    }
    variants = json.loads(os.environ.get("PROBE_VARIANTS", '{"ldsB": {}, "directB": {"RSLRL_X6_DIRECTB": "1"}}'))
    res = {"lib": os.environ.get("RSLRL_AMD_LIB", "default")}
    rounds = int(os.environ.get("PROBE_ROUNDS", 3))
    for name, fn in cases.items():
        r = {tag: [] for tag in variants}
        for _ in range(rounds):  # variants interleaved, min over rounds (clock drift)
            for tag, env in variants.items():
                for k, v in env.items():
                    os.environ[k] = v
                r[tag].append(t(fn))
                for k in env:
                    os.environ.pop(k)
        res[name] = {tag: min(v) for tag, v in r.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
