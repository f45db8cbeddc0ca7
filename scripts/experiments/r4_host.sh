# rollout host-time changes: record plan, cached Normal per act graph, env output ring -- tests, host split, shares
set -e
o=gpurun_out/r4/host
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_act_graph.py tests/test_gpu_update.py tests/test_gpu_env.py tests/test_gpu_minibatch.py tests/test_gpu_actor_head.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python scripts/rollout_host_split.py 16384 2>/dev/null | tail -1
for rep in 1 2; do
  timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 15 > $o/b16k_$rep.json 2> $o/b16k_$rep.err
  python -c "
import json; d=json.loads(open('$o/b16k_$rep.json').read().strip().splitlines()[-1])
print($rep, d['value'], d['ms_per_step'], d['phases_timed_ms']['collection'])"
done
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 10 > $o/c3.json 2> $o/c3.err
python -c "
import json; d=json.loads(open('$o/c3.json').read().strip().splitlines()[-1])
print('C3', d['value'], d['ms_per_step'], d['phases_timed_ms']['collection'][:5])"
# rollout_record: records per copy block (RSLRL_REC_ROWS build variants)
for v in default rec32 rec16; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 8 > $o/rec_$v.json 2> $o/rec_$v.err
  python -c "
import json; d=json.loads(open('$o/rec_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['hot_path']['kernels']['rollout_record'])"
done
# actor head: packed-FMA dW (default) vs the scalar 12-accumulator form (ah_s12)
for rep in 1 2; do
for v in default ah_s12; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/actor_head_probe.py --rounds 4 > $o/ah_${v}_$rep.json
  echo $v $(cat $o/ah_${v}_$rep.json)
done
done
