set -e
mkdir -p gpurun_out
for d in 1 2 3; do
  RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/x6d$d/librslrl_amd.so timeout -k 10 120 python scripts/x6_probe.py
done
