# rollout_record block order: per-env blocks on the low block indices (env_first) vs copy blocks first (default)
set -e
o=gpurun_out/r4/envfirst
mkdir -p $o
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/env_first/librslrl_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_plan.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2 3; do
for v in default env_first; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 6 --warmup 2 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v', $rep, d['value'], r['kernel'], r['mean_launch_us'], r['frac'])"
done
done
