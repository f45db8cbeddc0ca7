set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/bench_h3.json 2>gpurun_out/bench_h3.err
