"""compute_returns_slots (rollout_storage.py:127-149 + the update's slot array) in isolation: every form x launch kind,
on one storage set (hot: the inputs may sit in the 256 MB Infinity Cache) and rotated over enough sets that the bytes
between two uses of a set exceed the MALL (MALL-free).  Per-call HIP-event spans here; run under
`rocprofv3 --kernel-trace --stats` for the kernels' own durations (the phases run in the printed order).

    python scripts/gae_probe.py --n 65536 16384 --reps 40 --out gpurun_out/gae_probe.json
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import kernels  # noqa: E402

MALL = 256 << 20


def make_set(T, N, dev, g):
    v = torch.randn(T, N, 1, device=dev, generator=g)
    r = torch.randn(T, N, 1, device=dev, generator=g)
    d = (torch.rand(T, N, 1, device=dev, generator=g) < 0.02).to(torch.uint8)
    lv = torch.randn(N, 1, device=dev, generator=g)
    lp = torch.randn(T, N, 1, device=dev, generator=g)
    ret, adv = torch.empty_like(v), torch.empty_like(v)
    slots = torch.empty(T, N, 4, device=dev)
    return v, r, d, lv, ret, adv, lp, slots


def run(sets, reps, form, coop, sleep=1):
    old_f = kernels.debug_knob("gae_form", form)
    old_c = kernels.debug_knob("gae_coop", coop)
    old_s = kernels.debug_knob("gae_sleep", sleep)
    try:
        ev = []
        for i in range(reps):
            v, r, d, lv, ret, adv, lp, slots = sets[i % len(sets)]
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            kernels.compute_returns_slots(v, r, d, lv, 0.99, 0.95, ret, adv, lp, slots)
            e.record()
            ev.append((s, e))
        torch.cuda.synchronize()
        us = sorted(1000.0 * s.elapsed_time(e) for s, e in ev[2:])
    finally:
        kernels.debug_knob("gae_form", old_f)
        kernels.debug_knob("gae_coop", old_c)
        kernels.debug_knob("gae_sleep", old_s)
    return {"median_us": us[len(us) // 2], "p10_us": us[len(us) // 10], "min_us": us[0], "calls": len(us)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[65536, 16384])
    ap.add_argument("--t", type=int, default=24)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--forms", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--coop", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--sleep", type=int, nargs="+", default=[1])
    ap.add_argument("--out", default="gpurun_out/gae_probe.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    T = a.t
    out = {"T": T, "phases": []}
    for N in a.n:
        per_set = 37 * T * N + 4 * N  # one-launch algorithmic bytes
        k = max(2, -(-2 * MALL // per_set))  # > 2x the MALL between two uses of a set
        sets = [make_set(T, N, dev, g) for _ in range(k)]
        L = kernels._lib.lib()
        v, r, d, lv, ret, adv, lp, slots = sets[0]
        chosen = L.rslrl_compute_returns_slots_form(T, N, v.data_ptr(), r.data_ptr(), d.data_ptr(), lp.data_ptr(),
                                                    ret.data_ptr(), adv.data_ptr())
        for form, coop, sleep in [(f, c, z) for f in a.forms for c in a.coop for z in a.sleep]:
            if (form == 0 and (coop or sleep != a.sleep[0])) or (coop and sleep != a.sleep[0]):
                continue  # the knobs do not apply / one sleep setting for the cooperative launches
            if True:
                for mode, ss in (("hot", sets[:1]), ("rotated", sets)):
                    res = run(ss, a.reps, form, coop, sleep)
                    res.update(N=N, form_cap=form, coop=coop, sleep=sleep, mode=mode, sets=len(ss), bytes=per_set,
                               auto_form=chosen,
                               tbps_median=per_set / (res["median_us"] * 1e-6) / 1e12)
                    out["phases"].append(res)
                    print(json.dumps(res), flush=True)
        del sets
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
