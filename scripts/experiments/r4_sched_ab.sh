# LLVM AMDGPU scheduling strategy for the whole library (-mllvm -amdgpu-sched-strategy=max-ilp / max-memory-clause)
# against the default scheduler: the x6 GEMM probe at 393216 rows (fwd, dgrad) and the C3 bench, alternating
set -e
o=gpurun_out/r4/sched_ab
mkdir -p $o
for rep in 1 2; do
for v in default sched_max-ilp sched_max-memory-clause; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 200 python scripts/gemm_ab.py --variants default --rounds 3 --M 393216 > $o/gemm_${v}_$rep.json 2> $o/gemm_${v}_$rep.err
  echo "$v $rep $(tr '\n' ' ' < $o/gemm_${v}_$rep.json | cut -c1-400)"
done
done
for rep in 1 2; do
for v in default sched_max-ilp sched_max-memory-clause; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 10 --warmup 2 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['value'], d['ms_per_step'], d.get('roofline_mlp',{}).get('frac'))"
done
done
