# round-4 final rocprofv3 kernel stats of the headline bench command (kernel trace + stats only)
set -e
o=gpurun_out/r4f2
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
tail -c 400 $o/bench_stats.json
