# nontemporal record stores (default) vs plain (rec_plain) at the 16384-env share, where a whole rollout's records
# (151 MB) would fit the 256 MB Infinity Cache: rocprof stats of rollout_record and gather_records + the bench value
set -e
o=gpurun_out/r4/nt16k
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for v in default rec_plain; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s_${v}_$rep -o run -- \
      python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 10 > $o/b16k_${v}_$rep.json 2> $o/b16k_${v}_$rep.err
  RSLRL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 15 > $o/v16k_${v}_$rep.json 2> $o/v16k_${v}_$rep.err
  python3 - <<P
import csv, json
rows = list(csv.DictReader(open("$o/s_${v}_$rep/run_kernel_stats.csv")))
k = {r["Name"].split("(")[0].split("::")[-1].split("<")[0].strip(): float(r["AverageNs"]) / 1e3 for r in rows}
d = json.loads(open("$o/v16k_${v}_$rep.json").read().strip().splitlines()[-1])
print("$v", $rep, d["value"], "record", round(k.get("rollout_record_kernel", -1), 2), "gather", round(k.get("gather_records_kernel", -1), 2))
P
done
done
