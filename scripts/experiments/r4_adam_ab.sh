# Adam element-parallel (default) vs the per-tensor walk (adam_old): optimizer + update tests, then rocprof kernel
# stats of the 16384-env share for each library, alternating
set -e
o=gpurun_out/r4/adam_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_update.py tests/test_gpu_update_variants.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for v in default adam_old; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s_${v}_$rep -o run -- \
      python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 8 > $o/b16k_${v}_$rep.json 2> $o/b16k_${v}_$rep.err
  python3 - <<P
import csv, json
rows = list(csv.DictReader(open("$o/s_${v}_$rep/run_kernel_stats.csv")))
k = {r["Name"].split("(")[0].split("::")[-1]: float(r["AverageNs"]) / 1e3 for r in rows}
d = json.loads(open("$o/b16k_${v}_$rep.json").read().strip().splitlines()[-1])
print("$v", $rep, d["value"], "adam", round(k.get("adam_kernel", -1), 2), "grad_sq", round(k.get("grad_sq_kernel", -1), 2))
P
done
done
