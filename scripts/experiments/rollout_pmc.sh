# FETCH_SIZE / WRITE_SIZE passes over a short default bench (rollout_record traffic), each its own time-limited run.
set -e
out=gpurun_out/rpmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/bench_$c -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $out/bench_$c.json
done
