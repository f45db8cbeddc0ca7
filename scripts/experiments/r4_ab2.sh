set -e
out=gpurun_out/r4/ab2
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_actor_head.py tests/test_gpu_rollout.py tests/test_gpu_update.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/ah_mfma/librslrl_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_actor_head.py > $out/tests_mfma.log 2>&1 || { tail -30 $out/tests_mfma.log; exit 1; }
tail -2 $out/tests_mfma.log
for rep in 1 2; do
for v in default ah_v1 ah_mfma; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/actor_head_probe.py --rounds 4 > $out/${v}_$rep.json
  echo $v $(cat $out/${v}_$rep.json)
done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > $out/bench.json 2> $out/bench.err
python -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:200]); print(json.dumps(d['hot_path']['kernels']))"
