"""Per-kernel average of every counter in rocprofv3 counter_collection.csv files under a directory.
    python scripts/pmc_table.py gpurun_out/pmc [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0][-60:] + " grid=" + r.get("Grid_Size", "")
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k)
    for c, vals in sorted(v.items()):
        print(f"   {c:34s} n={len(vals):3d} avg={sum(vals) / len(vals):.4g}")
