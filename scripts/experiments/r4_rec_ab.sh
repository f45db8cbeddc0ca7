# rollout record: per-env scalars inside the record copy blocks (default) vs separate per-env blocks (rec_old)
set -e
o=gpurun_out/r4/rec_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_plan.py tests/test_gpu_act_graph.py tests/test_gpu_update.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for rep in 1 2; do
for v in default rec_old; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 8 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v', $rep, d['value'], r['kernel'], r['mean_launch_us'], r['frac'], r['call_span_us'])"
done
done
