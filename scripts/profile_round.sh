# Round profile capture on the GPU box (run from the repo root under gpurun; every GPU step time-limited):
#   1. rocprofv3 --kernel-trace --stats over the headline bench command  -> gpurun_out/prof/stats
#   2. FETCH_SIZE and WRITE_SIZE passes (separate: they do not fit one pass) over a short bench run
#   3. the same two passes over the 512 MiB calibration copy (scripts/pmc_calibration.py)
# Then, on the build host: scripts/pmc_summary.py -> profiles/<round>_pmc_traffic.json.
set -e
out=gpurun_out/prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $out/bench_stats.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/bench_$c -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $out/bench_$c.json
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/cal_$c -o run -- \
      python3 scripts/pmc_calibration.py > $out/cal_$c.log
done
