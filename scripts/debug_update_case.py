"""Run one single-rank update fixture (tests/golden/update_<case>.npz) on the GPU in each GEMM mode and print
per-parameter errors against the reference (diagnostic for tests/test_gpu_update_variants.py)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from update_fixtures import build_update, param_errors, run_recorded_update  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402

case, fam = sys.argv[1], sys.argv[2]
meta = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))[fam][case]
z = np.load(os.path.join(ROOT, f"tests/golden/update_{case}.npz"))
for mode in ("x6", "f32"):
    prev = fused_mlp.set_gemm_mode({"x6": fused_mlp.GEMM_X6, "f32": fused_mlp.GEMM_F32}[mode])
    alg, pol = build_update(z, "r0/", meta, meta["ranks"][0], "cuda:0")
    grads = [None]
    loss, lr = run_recorded_update(alg, grads)
    fused_mlp.set_gemm_mode(prev)
    print(mode, "lr equal", lr == meta["ranks"][0]["lr_trace"], "loss", loss, meta["ranks"][0]["loss_dict"])
    r = torch.from_numpy(z["r0/grad_mb0"]).double()
    print(mode, "grad0 err", ((grads[0].double() - r).abs().max() / r.abs().max()).item())
    e = param_errors(pol.state_dict(), z, "r0/")
    print(mode, {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in e.items()})
    print(mode, "sens", meta.get("ulp_sensitivity"))
    if "std" in dict(pol.named_parameters()):
        print("std ours", pol.std.detach().cpu().numpy())
        print("std ref ", z["r0/final/std"])
        print("std init", z["r0/init/std"])
