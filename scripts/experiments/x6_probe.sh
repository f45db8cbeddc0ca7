# A/B of the x6 kernels: the committed library build (variants/base) vs the working tree's, alternating
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in rsl_rl_amd/lib/variants/base/librslrl_amd.so rsl_rl_amd/lib/librslrl_amd.so; do
    RSLRL_AMD_LIB=$lib PROBE_ROUNDS=2 PROBE_VARIANTS='{"v": {}}' timeout -k 10 120 python scripts/x6_probe.py
  done
done
