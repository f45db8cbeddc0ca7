# Same-box A/B of the launch-bound loss-kernel events at the 16384-env share (RSLRL_BENCH_LAUNCH_EVENTS=0 vs 1).
set -e
mkdir -p gpurun_out/evab16
for r in 1 2; do
  for w in 0 1; do
    RSLRL_BENCH_LAUNCH_EVENTS=$w timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > gpurun_out/evab16/r${r}_$w.json 2> gpurun_out/evab16/r${r}_$w.err
  done
done
