set -e
o=gpurun_out/r4/host2
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_plan.py tests/test_gpu_rollout.py tests/test_gpu_act_graph.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python scripts/rollout_host_split.py 16384 2>/dev/null | tail -1
for rep in 1 2; do
  timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 15 > $o/b16k_$rep.json 2> $o/b16k_$rep.err
  python -c "
import json; d=json.loads(open('$o/b16k_$rep.json').read().strip().splitlines()[-1])
print($rep, d['value'], d['ms_per_step'], d['phases_timed_ms']['collection'])"
done
