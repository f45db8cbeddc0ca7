set -e
mkdir -p gpurun_out/r4
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/r4/bench_base.json 2> gpurun_out/r4/bench_base.err
bash scripts/mlp_pmc.sh gpurun_out/r4/mlppmc
