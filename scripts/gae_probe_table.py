"""Per-phase kernel durations of scripts/gae_probe.py from its rocprofv3 kernel trace (the phases run in the order the
probe's JSON lists them, each `reps` calls of compute_returns_slots: one kernel for the one-launch forms, scan + normaliser
for the two-launch form).

    python scripts/gae_probe_table.py gpurun_out/r6/gae_probe.json gpurun_out/r6/gae_prof/gae_kernel_trace.csv
"""
import csv
import json
import statistics
import sys

GAE = ("gae_scan_kernel", "adv_normalize_slots_kernel", "gae_fused_slots_kernel", "gae_staged_slots_kernel")


def main(probe_json, trace_csv, out=None):
    probe = json.load(open(probe_json))
    rows = [r for r in csv.DictReader(open(trace_csv)) if any(k in r["Kernel_Name"] for k in GAE)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    i = 0
    table = []
    for ph in probe["phases"]:
        calls = ph["calls"] + 2  # the probe drops 2 warm calls from its event statistics
        per_call = 2 if ph["form_cap"] == 0 else 1
        seg = rows[i:i + calls * per_call]
        i += calls * per_call
        durs = []
        names = set()
        for c in range(2, calls):
            ks = seg[c * per_call:(c + 1) * per_call]
            names.update(k["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1] for k in ks)
            durs.append(sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks) / 1e3)
        durs.sort()
        med = statistics.median(durs)
        ent = {k: ph[k] for k in ("N", "form_cap", "coop", "sleep", "mode", "sets", "bytes")}
        ent.update(kernels=sorted(names), kernel_median_us=round(med, 2), kernel_p10_us=round(durs[len(durs) // 10], 2),
                   hbm_frac_median=round(ph["bytes"] / (med * 1e-6) / 8e12, 3), span_median_us=round(ph["median_us"], 2))
        table.append(ent)
        print(f"N={ent['N']:6d} cap={ent['form_cap']} coop={ent['coop']} sleep={ent['sleep']} {ent['mode']:8s} "
              f"{'+'.join(ent['kernels']):45s} kernel {med:6.2f} us (p10 {ent['kernel_p10_us']:6.2f})  "
              f"frac {ent['hbm_frac_median']:.3f}  span {ent['span_median_us']:6.2f}")
    assert i == len(rows), (i, len(rows))
    if out:
        json.dump({"source": [probe_json, trace_csv], "bytes": "one-launch algorithmic bytes per call (37 T N + 4 N)",
                   "phases": table}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
