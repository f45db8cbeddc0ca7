# The deferred permutation prefetch: its tests, the update-start host probe, and benches at the share and C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6pf}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_minibatch.py tests/test_gpu_act_graph.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 300 python3 scripts/update_start_probe.py --num-envs 16384 --iters 6 --out $o/update_start.json 2>/dev/null
for r in 1 2; do
  for n in 16384 65536; do
    timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_r$r.json 2> $o/b${n}_r$r.err || { tail -20 $o/b${n}_r$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$o/b${n}_r$r.json'));print($n,'run',$r,d['value'],d['ms_per_step'])"
  done
done
