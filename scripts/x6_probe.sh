set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in rsl_rl_amd/lib/variants/base/librslrl_amd.so rsl_rl_amd/lib/librslrl_amd.so; do
    PROBE_DEEP_ONLY=1 RSLRL_AMD_LIB=$lib timeout -k 10 120 python scripts/x6_probe.py
  done
done
