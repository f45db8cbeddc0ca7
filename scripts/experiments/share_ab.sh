# Strong-scaling share (16384 envs on one GPU = N=8's per-GPU work): one vs two streams for the actor / critic
# launches of the update, each its own time-limited run.
set -e
mkdir -p gpurun_out/share
for ts in 0 1; do
  RSLRL_TWO_STREAMS=$ts timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 20 > gpurun_out/share/ts$ts.json 2> gpurun_out/share/ts$ts.err
done
