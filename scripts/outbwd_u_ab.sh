# A/B of the output-layer backward's rows in flight per wave (RSLRL_OUTBWD_U build variants, rsl_rl_amd/lib/variants/uN)
set -e
mkdir -p gpurun_out/uab
for rep in 1 2; do
  for v in base u8 u16; do
    if [ $v = base ]; then lib=rsl_rl_amd/lib/librslrl_amd.so; else lib=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
    RSLRL_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 10 > gpurun_out/uab/$v.$rep.json 2> gpurun_out/uab/$v.$rep.err
  done
done
