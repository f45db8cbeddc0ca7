set -e
out=gpurun_out/r4/staged2
rm -rf $out; mkdir -p $out /tmp/sd
for v in default noswz noslp unstaged; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/x.pt --M 98304 > $out/det_$v.txt 2>&1
done
rm -rf /tmp/sd
