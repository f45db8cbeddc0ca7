# Round-5 closing measurements (every GPU step time-limited; counters in their own passes):
#   the default bench line (with the CPU baseline), the N = 8 / N = 4 per-GPU shares, rocprofv3 kernel stats of the
#   headline command, FETCH_SIZE / WRITE_SIZE passes of a short bench run + the calibration copy, and the MLP counters
#   (scripts/mlp_pmc.sh, scripts/hidden_bwd_pmc.sh).  Summaries on the build host.
set -e
o=${1:-gpurun_out/r5final}
mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench_default.json 2> $o/bench_default.err
timeout -k 10 200 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k.json 2> $o/b16k.err
timeout -k 10 200 python bench.py --global-num-envs 32768 --no-extra --no-cpu-baseline --steps 10 > $o/b32k.json 2> $o/b32k.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $o/bench_$c -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $o/bench_$c.json 2> $o/bench_$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $o/cal_$c -o run -- \
      python3 scripts/pmc_calibration.py > $o/cal_$c.log 2>&1
done
bash scripts/mlp_pmc.sh $o/mlppmc
bash scripts/hidden_bwd_pmc.sh $o/hbpmc
