# Alternating A/B of two library builds (A: the in-tree librslrl_amd.so, B: $1 = a variant .so, e.g.
# rsl_rl_amd/lib/variants/X/librslrl_amd.so) on the GEMM probe and on bench.py; output dir $2.
set -e
B=$1
out=${2:-gpurun_out/lib_ab}
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 120 python scripts/gemm_ab.py --variants ${GV:-default} --rounds 3 > $out/gemm_a$rep.json 2>/dev/null
  RSLRL_AMD_LIB=$B timeout -k 10 120 python scripts/gemm_ab.py --variants ${GV:-default} --rounds 3 > $out/gemm_b$rep.json 2>/dev/null
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $out/bench_a$rep.json 2>/dev/null
  RSLRL_AMD_LIB=$B timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $out/bench_b$rep.json 2>/dev/null
done
