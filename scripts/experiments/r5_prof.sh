# Round-5 profiles (every GPU step time-limited; counters in their own passes, never with trace domains):
#   rocprofv3 --kernel-trace --stats of the headline bench command; FETCH_SIZE / WRITE_SIZE passes over a short bench
#   run and over the 512 MiB calibration copy; the MLP forward pair's and the fused hidden backward's SQ + traffic
#   counters (scripts/mlp_pmc.sh, scripts/hidden_bwd_pmc.sh).
# Summaries on the build host: scripts/pmc_summary.py, scripts/mlp_pmc_summary.py.
set -e
o=${1:-gpurun_out/r5prof}
mkdir -p $o
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
