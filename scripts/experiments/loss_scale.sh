# Loss-kernel time against mini-batch size (fixed per-launch cost = the intercept), MALL-free rotation.
set -e
for n in 65536 32768 16384; do
  echo "envs=$n"
  MICROBENCH_ENVS=$n timeout -k 10 120 python scripts/hotpath_microbench.py --only loss --iters 400
done
