"""Print the bench lines of an A/B directory: value, ms/step, phases."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.load(open(f))
    except ValueError:
        continue
    if "value" not in d:
        continue
    print(f"{os.path.basename(f):18s} {d['value']:>12.0f} {d['ms_per_step']:8.3f} ms  coll {d['phases_last_iter'].get('collection_time', 0)*1e3:6.2f} ms  "
          f"learn {d['phases_last_iter'].get('learn_time', 0)*1e3:7.2f} ms  mlp {((d.get('roofline_mlp') or {}).get('mlp_ms_per_step') or 0):7.2f}")
