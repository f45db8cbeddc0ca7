# strong-scaling share (16384 envs): per-iteration host phase times over repeated runs (collection-time variance), and
# an A/B of the batched fold's unroll (default 8 vs 16: rsl_rl_amd/lib/variants/fold16)
set -e
o=gpurun_out/r4/share_diag
mkdir -p $o
for rep in 1 2; do
  for v in default fold16; do
    if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
    RSLRL_AMD_LIB=$L timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 15 > $o/b16k_${v}_$rep.json 2> $o/b16k_${v}_$rep.err
    python -c "
import json; d=json.loads(open('$o/b16k_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['value'], d['ms_per_step'], d['phases_timed_ms'])"
  done
done
for v in default fold16; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 10 > $o/c3_$v.json 2> $o/c3_$v.err
  python -c "
import json; d=json.loads(open('$o/c3_$v.json').read().strip().splitlines()[-1])
print('C3 $v', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default fold16; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats16k_$v -o run -- \
    python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 5 --warmup 2 > $o/stats16k_$v.json 2> $o/stats16k_$v.err
done
python - <<'P'
import csv, glob
for v in ("default", "fold16"):
    for f in glob.glob(f"gpurun_out/r4/share_diag/stats16k_{v}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "fold_batch" in r["Name"]:
                print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
P
