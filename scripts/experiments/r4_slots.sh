set -e
out=gpurun_out/r4/slots
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_minibatch.py tests/test_gpu_gae.py tests/test_gpu_rollout.py tests/test_gpu_update.py tests/test_capi.py > $out/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > $out/bench.json 2> $out/bench.err
for rep in 1 2; do
  RSLRL_OUT_FWD_OCC=4 timeout -k 10 200 python bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-extra > $out/occ4_$rep.json 2>/dev/null
  RSLRL_OUT_FWD_OCC=2 timeout -k 10 200 python bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-extra > $out/occ2_$rep.json 2>/dev/null
done
