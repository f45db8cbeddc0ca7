# The fused hidden backward's partial rows written with nontemporal stores (RSLRL_HB_VARIANT=1,5) against the default:
# its parity test under the variant, rocprof of the share's bench both ways, bench A/B at the share and C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6hbnt}
mkdir -p $o
RSLRL_HB_VARIANT=1,5 timeout -k 10 300 python -u -m pytest tests/test_gpu_hidden_bwd.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for v in 1,0 1,5; do
  RSLRL_HB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats_${v/,/_} -o s16k -- python3 bench.py --global-num-envs 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > /dev/null 2>&1
done
echo stats done
for r in 1 2 3; do
  for v in 1,2 1,5; do
    for n in 16384 65536; do
      RSLRL_HB_VARIANT=$v timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b${n}_v${v/,/_}_r$r.json 2> $o/b${n}_r$r.err || { tail -20 $o/b${n}_r$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o/b${n}_v${v/,/_}_r$r.json'));print($n,'variant','$v','run',$r,d['value'],d['ms_per_step'])"
    done
  done
done
