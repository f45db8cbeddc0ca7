# rollout_mlp form 2 (two tiles per workgroup, one phase apart): parity, then the rollout-step A/B of the three paths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rm4}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
RSLRL_ROLLOUT_MLP_FORM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py -x -q --timeout 200 --timeout-method thread > $o/pytest_form1.log 2>&1 || { tail -30 $o/pytest_form1.log; exit 1; }
tail -1 $o/pytest_form1.log
timeout -k 10 300 python3 scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 240 --rounds 4 --modes 0 1 2 --out $o/ab.json > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
grep median $o/ab.log || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s -o s -- python3 scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 100 --rounds 1 --graph 0 --modes 1 2 --out $o/ab_prof.json > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
echo done
