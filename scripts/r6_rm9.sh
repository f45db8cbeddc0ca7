set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6rm9
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py tests/test_gpu_act_graph.py tests/test_gpu_pair.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6rm9/pytest.log 2>&1 || { tail -30 gpurun_out/r6rm9/pytest.log; exit 1; }
tail -1 gpurun_out/r6rm9/pytest.log
bash scripts/r6_rm_pmc.sh gpurun_out/r6rm9/pmc | tail -1
