"""Times the fused actor head (rslrl_actor_head_fwd_bwd) against the separate launches it replaces (fused output-layer
forward + PPO loss kernel + output-layer backward) at the update's mini-batch size, interleaved rounds in one process
(HIP events around each call).  RSLRL_AMD_LIB selects a diagnostic build (e.g. RSLRL_AH_NODW / RSLRL_AH_NODZ).

    python scripts/actor_head_probe.py [--M 393216] [--rounds 5] [--iters 10]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib, kernels  # noqa: E402
from rsl_rl_amd.networks import fused_mlp as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=393216)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M, K, N, A = args.M, 256, 256, 12
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x = torch.nn.functional.elu(r(M, K))
    w, b, wo, bo = r(N, K) / 16, r(N) * 0.1, r(A, N) / 16, r(A) * 0.1
    sigma = torch.rand(A, device=dev, generator=g) * 0.5 + 0.5
    old_sigma = sigma.expand(M, A).contiguous()
    acts, ologp, adv, tv, ret, omu, vals = r(M, A), r(M, 1) - 8, r(M, 1), r(M, 1), r(M, 1), r(M, A) * 0.1, r(M, 1)
    img, out_img, img_t = F.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT), (wo, True)])
    head = F.ActorHead(acts, ologp, adv, tv, ret, omu, old_sigma, sigma, clip_param=0.2, value_loss_coef=1.0,
                       entropy_coef=0.01, use_clipped=True, compute_kl=True, grad_sigma=torch.empty(A, device=dev),
                       stats=torch.empty(8, device=dev))
    head.values = vals

    def fused():
        assert F.actor_head_fwd_bwd(x, b, N, img, bo, out_img, img_t, head) is not None

    def separate():
        h, mu = F.linear_fwd_out_ex(x, b, N, img, _lib.ARITH_X6, None, bo, out_img, store_h=True)
        _, gmu, _, _ = kernels.ppo_loss_fwd_bwd(mu, sigma, vals, acts, ologp, adv, tv, ret, omu, old_sigma,
                                                compute_kl=True)
        F.linear_dgrad_elu_wgrad(gmu, wo, h, img_t)

    res = {"fused": [], "separate": []}
    for fn in (fused, separate):
        fn()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, fn in (("fused", fused), ("separate", separate)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1000.0 / args.iters)
    out = {k: {"median_us": round(statistics.median(v), 2), "runs_us": [round(t, 2) for t in v]} for k, v in res.items()}
    out["lib"] = os.environ.get("RSLRL_AMD_LIB", "default")
    out["M"] = M
    print(json.dumps(out))


if __name__ == "__main__":
    main()
