"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic per kernel.

    python scripts/pmc_summary.py --fetch DIR --write DIR [--calib-fetch DIR --calib-write DIR] -o profiles/X.json

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE
counts half of the bytes of a wide (16-B/lane) streaming read, WRITE_SIZE counts 16-B stores exactly.
The calibration pass (scripts/pmc_calibration.py: a 512 MiB copyBuffer) is used to verify both factors
on the box before they are applied: traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch.
"""

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SHORT = {
    "ppo_loss_kernel": "ppo_loss",
    "ppo_loss_quad_kernel": "ppo_loss",
    "gae_scan_kernel": "gae_scan",
    "gae_fused_slots_kernel": "compute_returns_one_launch",
    "gae_staged_slots_kernel": "compute_returns_one_launch",
    "adv_normalize_kernel": "adv_normalize",
    "adv_normalize_slot_kernel": "adv_normalize_slot",
    "adv_normalize_slots_kernel": "adv_normalize_slots",
    "mlp_gemm_x6_value_head_kernel": "x6_value_head",
    "mlp_gemm_x6_actor_head_kernel": "x6_actor_head",
    "hidden_bwd_kernel": "x6_hidden_bwd_pair",
    "fwd_stream_kernel": "x6_fwd_stream_pair",
    "rollout_mlp_kernel": "rollout_mlp_pair",
    "value_head_stream_kernel": "x6_value_head_stream",
    "out_bwd_valu_kernel": "out_bwd",
    "out_bwd_valu_pair_kernel": "out_bwd_pair",
    "moments_kernel": "moments",
    "gather_rows_kernel": "gather_rows",
    "gather_records_kernel": "gather_rows",
    "record_fill_slot_kernel": "record_fill_slot",
    "rollout_record_kernel": "rollout_record",
    "centered_sq_kernel": "adv_centered_sq",
    "rnd_update_kernel": "rnd_update",
    "rnd_fold_kernel": "rnd_fold",
    "synthetic_env_kernel": "synthetic_env",
    "fold_batch_kernel": "fold_batch",
    "normal_affine_kernel": "normal_affine",
    "mlp_gemm_x6_kernel<1": "x6_fwd_elu",
    "mlp_gemm_x6_kernel<2": "x6_dgrad_elu",
    "wgrad_x6_kernel": "x6_wgrad",
    "wgrad_fold_kernel": "wgrad_fold",
    "__amd_rocclr_copyBuffer": "copyBuffer",
}
# kernels launched at several shapes are keyed "<short>@grid=<threads>"
BY_GRID = {"x6_fwd_elu", "x6_fwd_elu_pair", "x6_dgrad_elu_pair_w4", "x6_fwd_elu_pair_w4", "x6_dgrad_elu_pair_w8",
           "x6_fwd_elu_pair_w8", "x6_dgrad_elu_pair", "x6_wgrad256_pair", "x6_fwd_out", "x6_fwd", "x6_dgrad_elu", "x6_wgrad", "wgrad_fold", "h3_fwd_elu", "h3_dgrad_elu", "h3_fwd_out",
           "x6_dgrad_wgrad", "h3_wgrad256", "x6_wgrad64", "x6_fwd_out", "x6_fwd_elu_pair", "h3_fwd_elu_pair"}


EPI_NAMES = {0: "fwd", 1: "fwd_elu", 2: "dgrad_elu", 3: "dgrad_wgrad", 4: "fwd_out"}


def gemm_name(kernel):
    """mlp_gemm_x6_kernel<EPI, FULL, MINW, NR, PL> / wgrad_x6_kernel<TN, FULL, PL>: arithmetic (PL 2 = h3,
    3 = x6) and epilogue in the key."""
    m = re.search(r"mlp_gemm_x6_kernel<(\d+), \w+, \d+, \d+, (\d+)[,>]", kernel)
    if m:
        return f"{'h3' if m.group(2) == '2' else 'x6'}_{EPI_NAMES.get(int(m.group(1)), m.group(1))}"
    m = re.search(r"mlp_gemm_x6_w([48])_pair_kernel<(\d+)>", kernel)
    if m:  # the 4-wave (128 x 64 per wave) and 256-row-tile layouts of the paired update GEMMs
        return f"x6_{EPI_NAMES.get(int(m.group(2)), m.group(2))}_pair_w{m.group(1)}"
    m = re.search(r"mlp_gemm_x6_pair_kernel<(\d+), \w+, (\d+)[,>]", kernel)
    if m:  # two problems per launch (grid y = 2): bytes per launch cover both
        return f"{'h3' if m.group(2) == '2' else 'x6'}_{EPI_NAMES.get(int(m.group(1)), m.group(1))}_pair"
    m = re.search(r"out_bwd_valu_kernel<(\d+), (\d+)>", kernel)
    if m:  # output-layer backward on the VALU, keyed by its reduction width
        return f"out_bwd_valu_nr{m.group(1)}"
    m = re.search(r"out_bwd_valu_pair_kernel<(\d+), \d+, (\d+), \d+>", kernel)
    if m:
        return f"out_bwd_valu_pair_nr{m.group(1)}_{m.group(2)}"
    m = re.search(r"mlp_gemm_x6_out_pair_kernel<\w+, \d+, (\d+), (\d+), \d+>", kernel)
    if m:
        return f"x6_fwd_out_pair_nr{m.group(1)}_{m.group(2)}"
    m = re.search(r"wgrad_x6_pair_kernel<(\d+), \w+, (\d+)", kernel)
    if m:
        return f"{'h3' if m.group(2) == '2' else 'x6'}_wgrad{m.group(1)}_pair"
    m = re.search(r"wgrad_x6_kernel<(\d+), \w+, (\d+)>", kernel)
    if m:
        return f"{'h3' if m.group(2) == '2' else 'x6'}_wgrad{m.group(1)}"
    if "fold_kernel" in kernel:
        return "wgrad_fold"
    return None


def load(d, counter):
    files = glob.glob(os.path.join(d, "*", "*_counter_collection.csv")) + glob.glob(
        os.path.join(d, "*_counter_collection.csv"))
    out = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = gemm_name(r["Kernel_Name"]) or next((v for k, v in SHORT.items() if k in r["Kernel_Name"]), None)
            if name:
                if name in BY_GRID:
                    name = f"{name}@grid={r['Grid_Size']}"
                out[name].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--num-envs", type=int, default=None, help="envs per GPU of the profiled bench command")
    ap.add_argument("--num-steps-per-env", type=int, default=24)
    args = ap.parse_args()
    res = {"units": "bytes per launch", "correction": "traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024"}
    if args.num_envs:  # bench.py reports this file's traffic only for the same workload
        res["workload"] = {"num_envs_per_gpu": args.num_envs, "num_steps_per_env": args.num_steps_per_env}
    if args.calib_fetch and args.calib_write:
        cf = load(args.calib_fetch, "FETCH_SIZE")["copyBuffer"]
        cw = load(args.calib_write, "WRITE_SIZE")["copyBuffer"]
        copy_bytes = 512 * 1024 * 1024
        res["calibration"] = {
            "copy_bytes": copy_bytes,
            "fetch_factor": copy_bytes / (sum(cf) / len(cf) * 1024),
            "write_factor": copy_bytes / (sum(cw) / len(cw) * 1024),
        }
    f = load(args.fetch, "FETCH_SIZE")
    w = load(args.write, "WRITE_SIZE")
    kern = {}
    for name in sorted(set(f) & set(w)):
        fk = sum(f[name]) / len(f[name])
        wk = sum(w[name]) / len(w[name])
        kern[name] = {"launches": len(f[name]), "FETCH_SIZE_KB": round(fk, 1), "WRITE_SIZE_KB": round(wk, 1),
                      "read_bytes": int(2 * fk * 1024), "write_bytes": int(wk * 1024),
                      "traffic_bytes": int((2 * fk + wk) * 1024)}
    res["kernels"] = kern
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
