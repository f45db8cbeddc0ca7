# Round 6: the RCCL collective at world 1 -- none / single / overlap A/B, then a kernel trace of none vs overlap
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6ov}
mkdir -p $o
timeout -k 10 400 python3 scripts/overlap_ab.py --num-envs 65536 16384 --iters 8 --rounds 3 --out $o/overlap_ab.json > $o/overlap_ab.log 2>&1 || { tail -30 $o/overlap_ab.log; exit 1; }
grep '"modes"' $o/overlap_ab.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o ov -- python3 scripts/overlap_ab.py --num-envs 16384 --iters 3 --rounds 1 --modes none overlap --out $o/overlap_trace_run.json > $o/overlap_trace.log 2>&1
echo trace rc=$?
