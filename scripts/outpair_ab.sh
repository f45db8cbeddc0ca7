# Rollout heads in one launch vs two (RSLRL_OUT_PAIR), 16384 envs, alternating runs on one box.
set -e
mkdir -p gpurun_out/opab
for r in 1 2; do
  for op in 0 1; do
    RSLRL_OUT_PAIR=$op timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 20 > gpurun_out/opab/r${r}_o$op.json 2> gpurun_out/opab/r${r}_o$op.err
  done
done
