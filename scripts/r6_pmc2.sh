# Round 6: PMC traffic summaries for the other SCALE workloads (32,768 envs = N 4's share, 131,072 = C4 on one GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6pmc}
mkdir -p $o
for c in FETCH_SIZE WRITE_SIZE; do
  for n in 32768 131072; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $o/b${n}_$c -o run -- python3 bench.py --global-num-envs $n --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $o/b${n}_$c.json 2> $o/b${n}_$c.err || { echo bench $n $c failed; tail -5 $o/b${n}_$c.err; exit 1; }
  done
done
echo pmc2 done
