# Kernel stats of the headline bench command (C3) for the per-iteration breakdown.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/c3prof && mkdir -p gpurun_out/c3prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/c3prof/bench.json 2> gpurun_out/c3prof/bench.err
