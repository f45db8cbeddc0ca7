set -e
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_update_variants.py tests/test_multi_rank_update.py > gpurun_out/r4/newtests.log 2>&1
