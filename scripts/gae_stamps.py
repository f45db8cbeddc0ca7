"""Phase timeline of compute_returns_slots' one-launch kernel (form 1) from the diagnostic stamps build
(RSLRL_GAE_STAMPS: s_memrealtime, 100 MHz, per block at 6 points; scripts/build_gae_variant.sh gaestamps
-DRSLRL_GAE_STAMPS).  Points: 0 start, 1 scan + moments done, 2 partial stored (and the returns' stores drained),
3 log-probs loaded, 4 statistics known (barrier passed), 5 advantages + slots stored.  The stamps' own vmcnt waits
serialise a little; read the phases, not the total.

    RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/gaestamps/librslrl_amd.so python scripts/gae_stamps.py
"""

from __future__ import annotations

import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib, kernels  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def main():
    L = _lib.lib()
    L.rslrl_gae_debug_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    kernels.debug_knob("gae_form", 1)
    for N in (65536, 32768, 16384):
        T = 24
        v = torch.randn(T, N, 1, device=dev, generator=g)
        r = torch.randn(T, N, 1, device=dev, generator=g)
        d = (torch.rand(T, N, 1, device=dev, generator=g) < 0.02).to(torch.uint8)
        lv = torch.randn(N, 1, device=dev, generator=g)
        lp = torch.randn(T, N, 1, device=dev, generator=g)
        ret, adv, slots = torch.empty_like(v), torch.empty_like(v), torch.empty(T, N, 4, device=dev)
        nb = -(-N // 256)
        runs = []
        for it in range(8):
            buf = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
            assert L.rslrl_gae_debug_stamps(buf.data_ptr()) == 0
            kernels.compute_returns_slots(v, r, d, lv, 0.99, 0.95, ret, adv, lp, slots)
            torch.cuda.synchronize()
            assert L.rslrl_gae_debug_stamps(None) == 0
            s = buf.view(nb, 8).cpu()
            t0 = int(s[:, 0].min())
            us = lambda x: (int(x) - t0) / 100.0  # noqa: E731  (100 MHz -> us)
            last = [b for b in range(nb) if int(s[b, 7]) == 1]
            ph = {}
            for k in range(6):
                col = [us(s[b, k]) for b in range(nb)]
                ph[f"p{k}"] = {"min": round(min(col), 2), "median": round(pct(col, 0.5), 2), "p90": round(pct(col, 0.9), 2),
                              "max": round(max(col), 2)}
            lb = last[0] if last else None
            runs.append({"phases_us_from_first_start": ph,
                         "last_block": lb, "last_block_stamps_us": [round(us(s[lb, k]), 2) for k in range(6)] if lb is not None else None})
        out[N] = runs[-1]
        out[N]["all_runs_end_max_us"] = [r["phases_us_from_first_start"]["p5"]["max"] for r in runs]
        print(N, json.dumps(out[N]), flush=True)
    kernels.debug_knob("gae_form", -1)
    os.makedirs("gpurun_out/r6", exist_ok=True)
    with open("gpurun_out/r6/gae_stamps.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
