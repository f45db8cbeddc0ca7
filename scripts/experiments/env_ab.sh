# Alternating A/B of bench.py under two environment settings at C3 and at the 16384-env share:
#   bash scripts/env_ab.sh "VAR=a" "VAR=b" OUTDIR
set -e
out=${3:-gpurun_out/env_ab}
mkdir -p $out
for rep in 1 2; do
  env $1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $out/c3_a$rep.json 2>/dev/null
  env $2 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $out/c3_b$rep.json 2>/dev/null
done
for rep in 1 2; do
  env $1 timeout -k 10 200 python bench.py --global-num-envs 16384 --steps 30 --warmup 3 --no-cpu-baseline --no-extra > $out/s16k_a$rep.json 2>/dev/null
  env $2 timeout -k 10 200 python bench.py --global-num-envs 16384 --steps 30 --warmup 3 --no-cpu-baseline --no-extra > $out/s16k_b$rep.json 2>/dev/null
done
