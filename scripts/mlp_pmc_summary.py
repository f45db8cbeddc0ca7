"""Summarise scripts/mlp_pmc.sh: per MLP GEMM pair kernel (average over its dispatches) the effective clock, MFMA
pipe utilisation, issue / wait split, LDS and VALU counts, and HBM traffic with FETCH_SIZE / WRITE_SIZE corrected by
factors calibrated on the box in the kernels' own access patterns (scripts/pmc_pattern_probe.hip: each calibration
kernel touches 512 MiB once, so factor = 512 MiB / (counter KiB * 1024)).

    python scripts/mlp_pmc_summary.py DIR [-o profiles/r4_mlp_pmc.json]

Counter units (MI355X_MICROARCH.md): FETCH_SIZE / WRITE_SIZE in KiB; GRBM_GUI_ACTIVE summed over the 8 XCDs (cycles x 8);
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles summed over waves; SQ_INSTS_MFMA instructions (each
v_mfma_f32_32x32x16_bf16 holds its SIMD's matrix pipe 32 cycles).
"""

from __future__ import annotations

import argparse
import csv
import json
import os
import re
from collections import defaultdict

CAL_BYTES = 512 << 20
SHORT = [
    (r"hidden_bwd_kernel", "x6_hidden_bwd_pair"),
    (r"fwd_stream_kernel", "x6_fwd_stream_pair"),
    (r"mlp_gemm_x6_w4_pair_kernel<2>", "x6_dgrad_pair_w4"),
    (r"mlp_gemm_x6_w4s_pair_kernel<2>", "x6_dgrad_pair_w4s"),
    (r"mlp_gemm_x6_pair_kernel<1,", "x6_fwd_elu_pair"),
    (r"mlp_gemm_x6_pair_kernel<2,", "x6_dgrad_pair"),
    (r"wgrad_x6_pair_kernel<256,", "x6_wgrad_pair"),
    (r"fold_wide_kernel", "fold_wide"),
    (r"read_v4", "cal_read_v4"),
    (r"read_gemm_a", "cal_read_gemm_a"),
    (r"read_c_b32", "cal_read_c_b32"),
    (r"write_c_b32_nt", "cal_write_c_b32_nt"),
    (r"write_v4", "cal_write_v4"),
]
# algorithmic HBM bytes per launch at M rows (both problems of a pair): what each kernel must move at least
ALGO = {
    "x6_fwd_elu_pair": lambda M: 2 * (M * 256 * 4 * 2),           # X read, H written
    "x6_fwd_stream_pair": lambda M: 2 * (M * 256 * 4 * 2),
    "x6_dgrad_pair_w4": lambda M: 2 * (M * 256 * 4 * 3),          # dZ, H read, dZ_prev written
    "x6_dgrad_pair_w4s": lambda M: 2 * (M * 256 * 4 * 3),
    "x6_dgrad_pair": lambda M: 2 * (M * 256 * 4 * 3),
    "x6_wgrad_pair": lambda M: 2 * (M * 256 * 4 * 2),             # dZ, H read (+ partials)
    # fused input + weight gradient (csrc/mlp_bwd_fused.hip): dZ, H read once, dZ_prev written, + 128 slice partial rows
    "x6_hidden_bwd_pair": lambda M: 2 * (M * 256 * 4 * 3 + min(128, M // 64) * 65792 * 4),
}
FLOPS = {k: (lambda M: 2 * 2 * M * 256 * 256) for k in ALGO}
FLOPS["x6_hidden_bwd_pair"] = lambda M: 2 * 2 * 2 * M * 256 * 256  # two GEMMs per problem
# which calibration pattern each kernel's traffic follows: (reads, writes)
PATTERN = {
    "x6_fwd_elu_pair": ("cal_read_gemm_a", "cal_write_c_b32_nt"),
    "x6_fwd_stream_pair": ("cal_read_v4", "cal_write_c_b32_nt"),
    "x6_dgrad_pair_w4": ("cal_read_gemm_a+cal_read_c_b32", "cal_write_c_b32_nt"),
    "x6_dgrad_pair": ("cal_read_gemm_a+cal_read_c_b32", "cal_write_c_b32_nt"),
    "x6_wgrad_pair": ("cal_read_v4", "cal_write_v4"),
    "x6_hidden_bwd_pair": ("cal_read_v4", "cal_write_c_b32_nt"),
}


def short(name):
    for pat, s in SHORT:
        if re.search(re.escape(pat) if "<" in pat else pat, name):
            return s
    return None


def read_pass(path):
    """{short: {counter: [value per dispatch]}}, {short: [duration ns per dispatch]}"""
    vals = defaultdict(lambda: defaultdict(dict))
    dur = defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            s = short(row["Kernel_Name"])
            if s is None:
                continue
            d = int(row["Dispatch_Id"])
            vals[s][row["Counter_Name"]][d] = vals[s][row["Counter_Name"]].get(d, 0.0) + float(row["Counter_Value"])
            dur[s][d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return vals, dur


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", "--out")
    ap.add_argument("--M", type=int, default=393216)
    args = ap.parse_args()
    d = args.dir
    counters = defaultdict(dict)
    durs = defaultdict(list)
    for p in ("sq1", "sq2", "mlp_FETCH_SIZE", "mlp_WRITE_SIZE", "cal_FETCH_SIZE", "cal_WRITE_SIZE"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        v, du = read_pass(f)
        for s, cs in v.items():
            for c, per in cs.items():
                counters[s][c] = mean(per.values())
        if p == "sq1":
            for s, per in du.items():
                durs[s] = list(per.values())
    cal = {}
    for s in ("cal_read_v4", "cal_read_gemm_a", "cal_read_c_b32"):
        if counters[s].get("FETCH_SIZE"):
            cal[s] = CAL_BYTES / (counters[s]["FETCH_SIZE"] * 1024)
    for s in ("cal_write_c_b32_nt", "cal_write_v4"):
        if counters[s].get("WRITE_SIZE"):
            cal[s] = CAL_BYTES / (counters[s]["WRITE_SIZE"] * 1024)
    kernels = {}
    M = args.M
    for s, c in counters.items():
        if s.startswith("cal_") or s not in ALGO:
            continue
        t_ns = mean(durs.get(s, [])) or None
        ent = {"launch_us_under_counters": round(t_ns / 1e3, 1) if t_ns else None}
        if c.get("GRBM_GUI_ACTIVE") and t_ns:
            clk = c["GRBM_GUI_ACTIVE"] / 8 / (t_ns * 1e-9)
            ent["clock_GHz"] = round(clk / 1e9, 3)
            if c.get("SQ_INSTS_MFMA"):
                # 1024 SIMDs, 32 cycles of a SIMD's matrix pipe per 32x32x16 bf16 MFMA
                ent["mfma_pipe_util"] = round(c["SQ_INSTS_MFMA"] * 32 / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 3)
        if c.get("SQ_WAVE_CYCLES"):
            w = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c and k != "SQ_BUSY_CYCLES":
                    ent[k.lower() + "_frac"] = round(c[k] / w, 3)
        for k in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_ACTIVE_INST_VALU", "SQ_VALU_MFMA_BUSY_CYCLES"):
            if k in c:
                ent[k] = c[k]
        algo = ALGO[s](M)
        ent["algorithmic_bytes"] = algo
        ent["flops_fp32_equiv"] = FLOPS[s](M)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rpat, wpat = PATTERN.get(s, ("cal_read_v4", "cal_write_v4"))
            rf = [cal.get(x) for x in rpat.split("+")]
            if all(rf) and cal.get(wpat):
                # reads of mixed patterns: the factors agree within a few % (checked below), their mean is applied
                f_read = sum(rf) / len(rf)
                traffic = c["FETCH_SIZE"] * 1024 * f_read + c["WRITE_SIZE"] * 1024 * cal[wpat]
                ent["traffic_bytes"] = int(traffic)
                ent["traffic_over_algorithmic"] = round(traffic / algo, 3)
                ent["read_factor"] = round(f_read, 4)
                ent["write_factor"] = round(cal[wpat], 4)
            ent["fetch_kib_raw"] = c["FETCH_SIZE"]
            ent["write_kib_raw"] = c["WRITE_SIZE"]
        kernels[s] = ent
    out = {"M": M, "calibration_factors": {k: round(v, 4) for k, v in cal.items()},
           "calibration_bytes_per_launch": CAL_BYTES, "kernels": kernels,
           "method": "scripts/mlp_pmc.sh + scripts/mlp_pmc_summary.py: traffic = FETCH_SIZE x read factor + WRITE_SIZE "
                     "x write factor, factors measured on the same box by kernels touching 512 MiB once in each GEMM's "
                     "own access pattern (scripts/pmc_pattern_probe.hip)"}
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
