set -e
out=gpurun_out/r4/ah_probe
mkdir -p $out
for v in default ah_nodw ah_nodz; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/actor_head_probe.py --rounds 4 > $out/$v.json
  cat $out/$v.json
done
