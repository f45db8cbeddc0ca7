# Kernel stats of the 16384-env share (N=8's per-GPU work) for the strong-scaling breakdown.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p16k2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p16k2 -o run -- python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/p16k2/bench.json 2> gpurun_out/p16k2/bench.err
