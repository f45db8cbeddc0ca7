# Round-end bench lines + rocprofv3 kernel stats, without the PMC passes (use round_final.sh when kernels changed:
# its profile_round.sh re-collects FETCH_SIZE / WRITE_SIZE).
set -e
o=gpurun_out/r3f2
mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench_default.json 2> $o/bench_default.err
timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k.json 2> $o/b16k.err
timeout -k 10 200 python bench.py --global-num-envs 32768 --no-extra --no-cpu-baseline --steps 10 > $o/b32k.json 2> $o/b32k.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
