# rollout_mlp cooperative per-chunk split (default build) vs every wave splitting on read (RSLRL_RM_COOP=0 variant):
# parity, then the rollout step per library in separate processes, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rm6}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for lib in rsl_rl_amd/lib/librslrl_amd.so rsl_rl_amd/lib/variants/rmsplit/librslrl_amd.so; do
    n=$(basename $(dirname $lib))
    RSLRL_AMD_LIB=$lib timeout -k 10 200 python3 scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 240 --rounds 1 --modes 1 --out $o/ab_${n}_$r.json > $o/ab_${n}_$r.log 2>&1 || { tail -20 $o/ab_${n}_$r.log; exit 1; }
    echo $n $r $(python3 -c "import json;d=json.load(open('$o/ab_${n}_$r.json'));print([x['one_launch']['median'] for x in d['runs']])")
  done
done
