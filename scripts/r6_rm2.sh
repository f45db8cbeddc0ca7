# rollout step A/B (scripts/rollout_mlp_ab.py) + rocprof stats of both forms at the 16,384-env share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rm2}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 300 python3 scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 240 --rounds 4 --out $o/ab.json > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
grep median $o/ab.log || true
for v in 0 1; do
  RSLRL_ROLLOUT_MLP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s$v -o s -- python3 scripts/rollout_mlp_ab.py --num-envs 16384 --steps 100 --rounds 1 --graph 0 --out $o/ab_prof$v.json > $o/prof$v.log 2>&1 || { tail -20 $o/prof$v.log; exit 1; }
done

for v in 0 1; do
  RSLRL_ROLLOUT_MLP=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/t$v -o t -- python3 bench.py --global-num-envs 16384 --steps 4 --warmup 2 --no-cpu-baseline --no-extra > $o/t$v.json 2> $o/t$v.err || { tail -20 $o/t$v.err; exit 1; }
done
echo traced
