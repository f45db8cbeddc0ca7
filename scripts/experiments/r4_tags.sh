set -e
o=gpurun_out/r4/tags
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_plan.py tests/test_gpu_loss.py tests/test_gpu_minibatch.py tests/test_gpu_rollout.py tests/test_capi.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline > $o/bench.json 2> $o/bench.err
python -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])); print(json.dumps(d['hot_path']['kernels']))"
# batched fold: 8 (default) vs 4 slices per load round at the 16384-env share (rocprof kernel stats)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default fold4; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats16k_$v -o run -- \
    python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 5 --warmup 2 > $o/stats16k_$v.json 2> $o/stats16k_$v.err
done
python - <<'P'
import csv, glob
for v in ("default", "fold4"):
    for f in glob.glob(f"gpurun_out/r4/tags/stats16k_{v}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "fold_batch" in r["Name"] or "rollout_record" in r["Name"]:
                print(v, r["Name"][:50], r["Calls"], r["AverageNs"])
P
