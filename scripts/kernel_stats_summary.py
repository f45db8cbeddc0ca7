"""Group a rocprofv3 kernel_stats.csv by kernel family and print per-step time shares.

    python scripts/kernel_stats_summary.py gpurun_out/prof/.../kernel_stats.csv --steps 7
    python scripts/kernel_stats_summary.py gpurun_out/prof/run_results.db --steps 7   (rocpd database)
"""

import argparse
import csv
import re

FAMILIES = [
    ("x6 gemm<fwd bias+ELU>", r"mlp_gemm_x6r?_kernel<1"),
    ("x6 gemm<fwd bias>", r"mlp_gemm_x6r?_kernel<0"),
    ("x6 gemm<dgrad ELU'>", r"mlp_gemm_x6r?_kernel<2"),
    ("x6 gemm<dgrad ELU' + wgrad>", r"mlp_gemm_x6_kernel<3"),
    ("x6 wgrad", r"wgrad_x6_kernel"),
    ("partials fold", r"wgrad_fold_kernel|fold_kernel<"),
    ("bimage", r"bimage_kernel"),
    ("f32 gemm<fwd bias+ELU>", r"mlp_gemm_kernel<1"),
    ("f32 gemm<fwd bias>", r"mlp_gemm_kernel<0"),
    ("f32 gemm<dgrad ELU'>", r"mlp_gemm_kernel<2"),
    ("colsum_fold", r"colsum_fold"),
    ("ppo_loss", r"ppo_loss_kernel"),
    ("gae_scan", r"gae_scan_kernel"),
    ("adv_normalize (+ record slots)", r"adv_normalize_kernel|adv_normalize_slot_kernel|moments_kernel"),
    ("x6 value head (fwd + d value loss + head bwd)", r"value_head_kernel"),
    ("gather_rows", r"gather_rows_kernel|gather_records_kernel"),
    ("record_fill_slot", r"record_fill_slot_kernel"),
    ("hipBLASLt GEMM", r"^Cijk_"),
    ("torch reduce", r"reduce_kernel"),
    ("torch multi_tensor (optimizer/clip)", r"multi_tensor_apply"),
    ("torch RNG", r"distribution_|normal_"),
    ("torch elementwise", r"elementwise_kernel|vectorized_"),
    ("copy/fill", r"__amd_rocclr"),
]


def rows(path):
    """(kernel name, total ns, calls) from a kernel_stats.csv or a rocpd .db."""
    if path.endswith(".db"):
        import sqlite3
        q = "select name, sum(duration), count(*) from kernels group by name"
        yield from sqlite3.connect(path).execute(q)
        return
    for r in csv.DictReader(open(path)):
        yield r["Name"], float(r["TotalDurationNs"]), int(r["Calls"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1, help="iterations covered by the trace")
    a = ap.parse_args()
    agg = {}
    total = 0.0
    for name, t, c in rows(a.csv):
        fam = next((f for f, p in FAMILIES if re.search(p, name)), "other: " + name[:60])
        e = agg.setdefault(fam, [0.0, 0])
        e[0] += t
        e[1] += c
        total += t
    print(f"{'family':40s} {'ms/step':>9s} {'calls/step':>10s} {'share':>6s}")
    for fam, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{fam:40s} {t / 1e6 / a.steps:9.3f} {c / a.steps:10.1f} {100 * t / total:5.1f}%")
    print(f"{'total busy':40s} {total / 1e6 / a.steps:9.3f}")


if __name__ == "__main__":
    main()
