# Round 6: per-workload HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes, never with trace domains) of the bench
# at C3 (65,536 envs) and at the N = 8 share (16,384 envs), plus the 512 MiB copy calibration; summaries per workload
# (scripts/pmc_summary.py --num-envs) are what bench.py's roofline.traffic reads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6pmc}
mkdir -p $o
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $o/cal_$c -o run -- python3 scripts/pmc_calibration.py > $o/cal_$c.log 2>&1 || { echo cal $c failed; tail -5 $o/cal_$c.log; exit 1; }
  for n in 65536 16384; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $o/b${n}_$c -o run -- python3 bench.py --global-num-envs $n --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $o/b${n}_$c.json 2> $o/b${n}_$c.err || { echo bench $n $c failed; tail -5 $o/b${n}_$c.err; exit 1; }
  done
done
echo pmc done
