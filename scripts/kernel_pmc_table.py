"""Clock, MFMA-pipe use and wait fractions of one kernel's dispatches from two rocprofv3 --pmc passes (sq1: SQ_WAVE_CYCLES
SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT; sq2:
SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD
SQ_INSTS_VMEM_WR); scripts/fs_pmc_table.py's arithmetic for any kernel.

    python scripts/kernel_pmc_table.py DIR KERNEL_SUBSTRING [MIN_US]
"""
import collections
import csv
import glob
import json
import sys

d0, name = sys.argv[1], sys.argv[2]
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
res = {}
for d in ("sq1", "sq2"):
    f = glob.glob(f"{d0}/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f)):
        if name not in r["Kernel_Name"]:
            continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    big = [i for i in agg if dur[i] >= min_us * 1e3]
    for k in agg[big[0]]:
        res[k] = sum(agg[i][k] for i in big) / len(big)
    res[d + "_us"] = sum(dur[i] for i in big) / len(big) / 1e3
    res[d + "_dispatches"] = len(big)
clk = res["GRBM_GUI_ACTIVE"] / 8 / (res["sq1_us"] * 1e-6)
print(json.dumps({"kernel": name, "dispatches": res["sq1_dispatches"], "us": round(res["sq1_us"], 1),
                  "clock_GHz": round(clk / 1e9, 3),
                  "mfma_pipe_util": round(res["SQ_INSTS_MFMA"] * 32 / (1024 * res["GRBM_GUI_ACTIVE"] / 8), 3),
                  "wait_any": round(res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"], 3),
                  "wait_inst": round(res["SQ_WAIT_INST_ANY"] / res["SQ_WAVE_CYCLES"], 3),
                  "active_inst": round(res["SQ_ACTIVE_INST_ANY"] / res["SQ_WAVE_CYCLES"], 3),
                  "valu_per_mfma": round(res["SQ_INSTS_VALU"] / res["SQ_INSTS_MFMA"], 2),
                  "lds_per_mfma": round(res["SQ_INSTS_LDS"] / res["SQ_INSTS_MFMA"], 2),
                  "lds_bank_conflict_per_lds_inst": round(res["SQ_LDS_BANK_CONFLICT"] / max(res["SQ_INSTS_LDS"], 1), 3)}))
