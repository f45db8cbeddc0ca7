"""rslrl_fold_partials_batch in isolation on the update's job sets (one mini-batch's weight-gradient folds): C3 and the
16,384-env share -- the four hidden-layer folds (128 slices x 65,792), the actor head's per-tile partials (tiles x 3,084),
the value head's slice rows (256 x 260) and the two first-layer folds (256 x 12,544).  HIP-event time per launch and the
bandwidth of the partials read.  Several libraries can be compared in one call (--libs a.so b.so: one child process
each, alternated).

    python scripts/fold_probe.py --reps 50 --out gpurun_out/fold_probe.json
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(reps):
    sys.path.insert(0, ROOT)
    import torch

    from rsl_rl_amd import _lib

    L = _lib.lib()
    dev = torch.device("cuda:0")
    out = {}
    for name, tiles in (("c3", 3072), ("share16k", 768)):
        specs = [(128, 65792)] * 4 + [(tiles, 3084), (256, 260), (256, 12544), (256, 12544)]
        g = torch.Generator(device=dev).manual_seed(0)
        parts = [torch.randn(S, NK, device=dev, generator=g) for S, NK in specs]
        outs = [torch.empty(NK, device=dev) for _, NK in specs]
        jobs = [_lib.FoldJob(p.data_ptr(), S, NK, o.data_ptr(), NK, 0, 0) for p, o, (S, NK) in zip(parts, outs, specs)]
        arr = (_lib.FoldJob * len(jobs))(*jobs)
        nbytes = L.rslrl_fold_partials_batch_workspace_bytes(arr, len(jobs))
        ws = torch.zeros(max(nbytes, 256) // 8 + 32, dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream().cuda_stream

        def call():
            _lib.check(L.rslrl_fold_partials_batch(arr, len(jobs), ws.data_ptr(), ws.numel() * 8, st), "fold")

        for _ in range(5):
            call()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            call()
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
        rd = sum(S * NK * 4 for S, NK in specs)
        for o, p in zip(outs, parts):
            ref = p.double().sum(0)
            assert float((o.double() - ref).abs().max()) <= 1e-6 * float(ref.abs().max()) + 1e-6
        out[name] = {"us": round(us, 2), "partials_MB": round(rd / 1e6, 1), "GB_s": round(rd / us / 1e3, 1)}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--libs", nargs="*", default=[])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--out", default="gpurun_out/fold_probe.json")
    a = ap.parse_args()
    if a.child or not a.libs:
        res = run_one(a.reps)
        if not a.child:
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            json.dump(res, open(a.out, "w"), indent=1)
        return
    res = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in (a.libs if r % 2 == 0 else a.libs[::-1]):
            env = dict(os.environ, RSLRL_AMD_LIB=lib)
            p = subprocess.run([sys.executable, __file__, "--child", "--reps", str(a.reps)], env=env, cwd=ROOT,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout + p.stderr, flush=True)
                raise SystemExit(1)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
            res[lib].append(json.loads(line))
            print(lib, line, flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
