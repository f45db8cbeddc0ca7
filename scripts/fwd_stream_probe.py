"""Median launch time of the update's square hidden-layer forward pair (x6, M = 393,216 and the rollout's 65,536) in
this process: RSLRL_FWD_STREAM=0 / 1 (read once per process) picks the tiled or the streaming kernel.  Run two
processes on one box for an A/B; under rocprofv3 for counters."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    out = {}
    shapes = [(393216, 256), (196608, 256), (98304, 256), (65536, 256), (16384, 256)]
    for M, K in shapes:
        g = torch.Generator(device=dev).manual_seed(1)
        xs = [torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g)) for _ in range(2)]
        ws = [torch.randn(256, K, device=dev, generator=g) / 16 for _ in range(2)]
        bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(2)]
        imgs = fused_mlp.bimages([(w, False, _lib.BIMAGE_LAYOUT_GEMM) for w in ws])
        ts = []
        for it in range(iters + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fused_mlp.linear_fwd_pair(xs, bs, 256, True, imgs, _lib.ARITH_X6, [None, None], [False, False])
            e1.record()
            torch.cuda.synchronize()
            if it >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        out[f"{M}x{K}"] = {"median_us": round(ts[len(ts) // 2], 1), "min_us": round(ts[0], 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
