# Loss-kernel grid sweep on the GPU box, MALL-free (4 rotated ~104 MB mini-batches), rollout-like old sigma.
set -e
mkdir -p gpurun_out
for b in 256 512 768 1024; do
  echo "blocks=$b"
  RSLRL_LOSS_QUAD_MAX_BLOCKS=$b timeout -k 10 120 python scripts/hotpath_microbench.py --only loss --iters 400
done
echo "kl_fast=0 blocks=256"
RSLRL_KL_FAST=0 timeout -k 10 120 python scripts/hotpath_microbench.py --only loss --iters 400
