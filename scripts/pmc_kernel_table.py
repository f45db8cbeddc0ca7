"""Mean PMC counter values per kernel name from rocprofv3 counter_collection CSVs (any number of pass dirs).

    python scripts/pmc_kernel_table.py gpurun_out/x6pmc/p1 gpurun_out/x6pmc/p2 [--filter substr]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
        args = [a for a in args if a != filt]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-90:]
                if filt and filt not in name:
                    continue
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-90:]
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, cs in acc.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        if dur.get(k):
            row["mean_us"] = sum(dur[k]) / len(dur[k])
        w = row.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in row:
                    row[c + "_frac"] = round(row[c] / w, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and "GRBM_GUI_ACTIVE" in row:
            # MFMA busy cycles summed over SIMDs (1024) vs GPU-active cycles
            row["mfma_busy_frac"] = round(row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        out[k] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
