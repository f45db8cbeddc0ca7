# The XCD-interleaved first-layer forward pair: its test, rocprof of the two grids alternated in one process, then
# bench A/B (RSLRL_PAIR_XCD=0 / 1) at C3 and the share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6xcd}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for f in 0 1; do
    for n in 65536 16384; do
      RSLRL_PAIR_XCD=$f timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_f${f}_r$r.json 2> $o/b${n}_f${f}_r$r.err || { tail -20 $o/b${n}_f${f}_r$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o/b${n}_f${f}_r$r.json'));print($n,'xcd',$f,'run',$r,d['value'],d['ms_per_step'],d['update_env_steps_per_s'])"
    done
  done
done
RSLRL_PAIR_XCD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats1 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > /dev/null 2>&1
RSLRL_PAIR_XCD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats0 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > /dev/null 2>&1
echo stats done
