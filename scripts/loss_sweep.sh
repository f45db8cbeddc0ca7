# Loss-kernel A/B on the GPU box: pipeline depth x grid size, MALL-free (4 rotated ~104 MB mini-batches).
set -e
mkdir -p gpurun_out
for d in 1 2 3; do
  for b in 256 512; do
    echo "depth=$d blocks=$b"
    RSLRL_LOSS_DEPTH=$d RSLRL_LOSS_QUAD_MAX_BLOCKS=$b timeout -k 10 120 python scripts/hotpath_microbench.py --only loss --iters 400
  done
done
