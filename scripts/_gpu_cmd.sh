set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_update.py -x -q --timeout 120 --timeout-method thread > gpurun_out/loss_tests.log 2>&1
timeout -k 10 120 python scripts/hotpath_microbench.py --only loss,loss_perrow --iters 200 > gpurun_out/mb_auto.json
RSLRL_LOSS_KERNEL=lane timeout -k 10 120 python scripts/hotpath_microbench.py --only loss,loss_perrow --iters 200 > gpurun_out/mb_lane.json
