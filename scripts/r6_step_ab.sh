# Same-box A/B of the rollout step fusion (the Normal sample inside the one-launch forward, the single-network
# one-launch forward of compute_returns' last values, copy-free act graphs for recurring observation buffers):
# RSLRL_ROLLOUT_STEP_FUSION=0 / 1 alternated, benches at the 16,384-env share and at C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6stepab}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_mlp.py tests/test_gpu_act_graph.py tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for f in 0 1; do
    for n in 16384 65536; do
      RSLRL_ROLLOUT_STEP_FUSION=$f timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_f${f}_r$r.json 2> $o/b${n}_f${f}_r$r.err || { tail -20 $o/b${n}_f${f}_r$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o/b${n}_f${f}_r$r.json'));print($n,'fusion',$f,'run',$r,d['value'],d['ms_per_step'])"
    done
  done
done
