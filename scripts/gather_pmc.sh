# Record vs per-field gather: alternating bench A/B, then one FETCH_SIZE / WRITE_SIZE pass per layout over a
# short bench run (each its own rocprofv3 run; the pmc counters of one block fit one pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/ab_bench.sh RSLRL_RECORD_LAYOUT=1 RSLRL_RECORD_LAYOUT=0
out=gpurun_out/gpmc
mkdir -p $out
for lay in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RSLRL_RECORD_LAYOUT=$lay timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/l${lay}_$c -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $out/l${lay}_$c.json
  done
done
