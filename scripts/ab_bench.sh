# Alternating A/B of bench.py under two environment settings (args: "ENV=VAL" for A, "ENV=VAL" for B)
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  env $1 timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/ab/a$rep.json 2>/dev/null
  env $2 timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/ab/b$rep.json 2>/dev/null
done
