# Round 6: the fused hidden backward variants -- interleaved MFMA chains (RSLRL_HB_VARIANT 1,5 / 1,6) and the reordered
# halves (1,7 .. 1,10) -- bit-exactness, then kernel time against the default (1,2 = prio) in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6hb}; mkdir -p $o
for v in 1,5 1,7 1,8; do
  RSLRL_HB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hidden_bwd.py -m gpu > $o/t_$v.log 2>&1 || { echo variant $v; tail -30 $o/t_$v.log; exit 1; }
  echo $v $(tail -1 $o/t_$v.log)
done
PROBE_ROUNDS=4 timeout -k 10 400 python3 scripts/hidden_bwd_probe.py --variants 1:2,1:5,1:6,1:7,1:8,1:9,1:10 > $o/probe.json 2> $o/probe.err || { tail -20 $o/probe.err; exit 1; }
cat $o/probe.json
