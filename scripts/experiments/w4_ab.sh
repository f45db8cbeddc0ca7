# Bench A/B of the w4 input-gradient layout (RSLRL_W4=0 vs default) at C3, alternating runs on one box.
set -e
mkdir -p gpurun_out/w4ab
for r in 1 2; do
  for w in 0 d; do
    if [ $w = 0 ]; then export RSLRL_W4=0; else unset RSLRL_W4; fi
    timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --steps 15 > gpurun_out/w4ab/r${r}_$w.json 2> gpurun_out/w4ab/r${r}_$w.err
  done
done
