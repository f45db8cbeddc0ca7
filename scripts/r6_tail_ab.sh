# The per-mini-batch tail inside the clip-and-Adam norm launch: its tests (+ the update fixtures that pin the lr
# trace), then RSLRL_FUSED_TAIL=0 / 1 alternated at the 16,384-env share and C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6tail}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_update_c3.py tests/test_gpu_update.py tests/test_gpu_update_variants.py tests/test_multi_rank_update.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for f in 0 1; do
    for n in 16384 65536; do
      RSLRL_FUSED_TAIL=$f timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_f${f}_r$r.json 2> $o/b${n}_f${f}_r$r.err || { tail -20 $o/b${n}_f${f}_r$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o/b${n}_f${f}_r$r.json'));print($n,'fused_tail',$f,'run',$r,d['value'],d['ms_per_step'])"
    done
  done
done
