# A/B of the library built without SLP (packed-f32) vectorisation (rsl_rl_amd/lib/variants/noslpall) against the
# shipped build: bench.py at C3 and at the N = 8 share, three alternating rounds on one box.
set -e
o=${1:-gpurun_out/noslp}
mkdir -p $o
for rep in 1 2 3; do
  for v in main noslpall; do
    if [ $v = main ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
    RSLRL_AMD_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
    RSLRL_AMD_LIB=$L timeout -k 10 200 python3 bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/s16_${v}_$rep.json 2> $o/s16_${v}_$rep.err
  done
done
