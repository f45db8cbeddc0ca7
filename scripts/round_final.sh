set -e
mkdir -p gpurun_out/r3f
timeout -k 10 400 python bench.py > gpurun_out/r3f/bench_default.json 2> gpurun_out/r3f/bench_default.err
timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > gpurun_out/r3f/b16k.json 2> gpurun_out/r3f/b16k.err
timeout -k 10 200 python bench.py --global-num-envs 32768 --no-extra --no-cpu-baseline --steps 10 > gpurun_out/r3f/b32k.json 2> gpurun_out/r3f/b32k.err
bash scripts/profile_round.sh
