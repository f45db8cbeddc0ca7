# Loss-kernel A/B on the GPU box (MALL-free: 4 rotated ~104 MB mini-batches, rollout-like old sigma): pipeline depth
# and grid size.
set -e
mkdir -p gpurun_out
for cfg in "1 256" "2 256" "1 512"; do
  set -- $cfg
  echo "depth=$1 blocks=$2"
  RSLRL_LOSS_DEPTH=$1 RSLRL_LOSS_QUAD_MAX_BLOCKS=$2 timeout -k 10 120 python scripts/hotpath_microbench.py --only loss --iters 400
done
