# The fused sample / single-network forward / direct act graphs: their GPU tests, then benches at the 16,384-env share
# and C3 alternated with RSLRL_ACT_DIRECT-free A/B is not available (the change is structural), so against the r6_final4
# numbers of the previous build on another box plus the kernel trace of the share.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6direct}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py tests/test_gpu_act_graph.py tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for n in 16384 65536; do
  timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b$n.json 2> $o/b$n.err || { tail -20 $o/b$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o/b$n.json'));print($n,d['value'],d['ms_per_step'],d['update_env_steps_per_s'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o s16k -- python3 bench.py --global-num-envs 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
echo stats rc=$?
