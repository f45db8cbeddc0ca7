"""Per-iteration GPU timeline of a bench kernel trace (rocprofv3 --kernel-trace csv): for each training iteration, the
rollout (first synthetic_env .. the GAE kernel) and the update (the record gather .. the last Adam) -- span, kernel busy
time and idle gaps -- and the top kernels of each phase.

    python scripts/trace_phases.py gpurun_out/r6share/trace/b16k_kernel_trace.csv
"""
import collections
import csv
import sys


def short(n):
    for p in ("void ", "rslrl::", "(anonymous namespace)::", "at::native::"):
        n = n.replace(p, "")
    return n.split("(")[0][:70]


def busy(ks):
    iv = sorted((k[0], k[1]) for k in ks)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(path, top=12):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
            for r in csv.DictReader(open(path))]
    rows.sort()
    gae = [i for i, r in enumerate(rows) if r[2].startswith("gae_")]
    iters = []
    for gi in gae:
        # rollout: back from the GAE kernel to the first synthetic_env after the previous update's last adam
        j = gi
        while j > 0 and not rows[j - 1][2].startswith("adam_kernel"):
            j -= 1
        k = gi + 1
        while k < len(rows) and not rows[k][2].startswith("gather_records"):
            k += 1
        e = k
        while e + 1 < len(rows) and not rows[e + 1][2].startswith("synthetic_env"):
            e += 1
        iters.append((rows[j:gi + 1], rows[k:e + 1]))
    for n, (roll, upd) in enumerate(iters):
        for name, ks in (("rollout", roll), ("update", upd)):
            if not ks:
                continue
            span = max(k[1] for k in ks) - ks[0][0]
            b = busy(ks)
            print(f"iter {n} {name:8s} span {span / 1e3:8.1f} us  busy {b / 1e3:8.1f} us  idle {(span - b) / 1e3:7.1f} us  "
                  f"kernels {len(ks)}")
    roll, upd = iters[-1]
    for name, ks in (("rollout", roll), ("update", upd)):
        c = collections.defaultdict(lambda: [0, 0])
        for s, e, nm in ks:
            c[nm][0] += e - s
            c[nm][1] += 1
        print(f"--- last iteration {name}: top kernels (total us, launches)")
        for nm, (t, cnt) in sorted(c.items(), key=lambda x: -x[1][0])[:top]:
            print(f"  {t / 1e3:9.1f} {cnt:5d}  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
