# rollout_record: where the time over a plain copy goes -- diagnostic builds (make HIPFLAGS+=-DRSLRL_REC_DIAG=v OUT=../lib/variants/recdiagv:
# 1 no log-prob, 2 no per-env blocks, 3 neither; wrong results, timing only) against the default, plus the plain-copy ceiling
set -e
o=gpurun_out/r4/rec_diag
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/cc -o cc -- python3 scripts/copy_ceiling.py > $o/cc_plan.json 2>$o/cc.err
for v in rec128 rec256; do RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/$v/librslrl_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_plan.py > $o/tests_$v.log 2>&1 || { tail -20 $o/tests_$v.log; exit 1; }; tail -1 $o/tests_$v.log; done
for rep in 1 2; do
for v in default recdiag1 recdiag2 recdiag3 rec128 rec256; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 6 --warmup 2 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v', $rep, d['value'], r['kernel'], r['mean_launch_us'], r['frac'], r['call_span_us'])"
done
done
