# Round-5 closing refresh after the host-side change (PPO.update without the start-of-update sync): the default bench
# line, the N = 8 / N = 4 shares and the rocprof kernel stats of the headline command (kernels unchanged since
# scripts/r5_final.sh, whose PMC passes stand).
set -e
o=${1:-gpurun_out/r5refresh}
mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench_default.json 2> $o/bench_default.err
timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k.json 2> $o/b16k.err
timeout -k 10 200 python bench.py --global-num-envs 32768 --no-extra --no-cpu-baseline --steps 10 > $o/b32k.json 2> $o/b32k.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
