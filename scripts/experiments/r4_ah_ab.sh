set -e
out=gpurun_out/r4/ah_ab
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_actor_head.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
for v in default ah_v1; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/actor_head_probe.py --rounds 4 > $out/${v}_$rep.json
  echo $v $(cat $out/${v}_$rep.json)
done
done
