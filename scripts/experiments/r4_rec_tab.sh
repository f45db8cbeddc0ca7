# rollout_record: log-prob sum through DPP quad broadcasts, one barrier (default) vs the LDS sum after a second barrier (rec_old)
set -e
o=gpurun_out/r4/rec_dpp
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_plan.py tests/test_gpu_update.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2 3 4; do
for v in default rec_old; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 6 --warmup 2 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v', $rep, d['value'], r['kernel'], r['mean_launch_us'], r['frac'], r['call_span_us'])"
done
done
