# Bench A/B of the launch-bound loss-kernel events (RSLRL_BENCH_LAUNCH_EVENTS=0 vs default), alternating on one box.
set -e
mkdir -p gpurun_out/evab
for r in 1 2; do
  for w in 0 1; do
    RSLRL_BENCH_LAUNCH_EVENTS=$w timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/evab/r${r}_$w.json 2> gpurun_out/evab/r${r}_$w.err
  done
done
