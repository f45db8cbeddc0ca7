"""Compare two scripts/value_head_probe.py dumps (tiled vs streaming head): max relative differences."""
import json
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
out = {}
for k in ("y", "dz", "dwb"):
    d = (a[k].double() - b[k].double()).abs().max().item()
    out[k] = {"max_abs": d, "rel_to_max": d / (a[k].double().abs().max().item() + 1e-30)}
out["dz_sum"] = [a["dz_sum"], b["dz_sum"]]
out["rows"] = [a["rows"], b["rows"]]
print(json.dumps(out))
