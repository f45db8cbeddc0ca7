"""Counters of the streaming forward's M = 393,216 dispatches (scripts/fwd_stream_ab.sh): clock, MFMA pipe use, waits."""
import collections
import csv
import glob
import sys

d0 = sys.argv[1]
res = {}
for d in ("sq1", "sq2"):
    f = glob.glob(f"{d0}/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f)):
        if "fwd_stream" not in r["Kernel_Name"]:
            continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    big = [i for i in agg if dur[i] > 300000]
    for k in agg[big[0]]:
        res[k] = sum(agg[i][k] for i in big) / len(big)
    res[d + "_us"] = sum(dur[i] for i in big) / len(big) / 1e3
clk = res["GRBM_GUI_ACTIVE"] / 8 / (res["sq1_us"] * 1e-6)
print({"us": round(res["sq1_us"], 1), "clock_GHz": round(clk / 1e9, 3),
       "mfma_util": round(res["SQ_INSTS_MFMA"] * 32 / (1024 * res["GRBM_GUI_ACTIVE"] / 8), 3),
       "wait_any": round(res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"], 3),
       "wait_inst": round(res["SQ_WAIT_INST_ANY"] / res["SQ_WAVE_CYCLES"], 3),
       "active_inst": round(res["SQ_ACTIVE_INST_ANY"] / res["SQ_WAVE_CYCLES"], 3),
       "valu_per_mfma": round(res["SQ_INSTS_VALU"] / res["SQ_INSTS_MFMA"], 2),
       "lds_per_mfma": round(res["SQ_INSTS_LDS"] / res["SQ_INSTS_MFMA"], 2)})
