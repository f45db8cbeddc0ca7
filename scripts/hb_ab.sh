# A/B of fused hidden-backward builds (rsl_rl_amd/lib/variants/<v>/librslrl_amd.so; "main" = the in-tree library):
# scripts/hidden_bwd_probe.py at 393,216 rows per build, alternating, each line beside its own separate-launch reference.
out=${1:-gpurun_out/hbab}
mkdir -p $out
for rep in 1 2; do
  for v in ${HB_VARIANTS:-main hbA hbBase}; do
    if [ $v = main ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
    RSLRL_AMD_LIB=$L timeout -k 10 120 python -u scripts/hidden_bwd_probe.py --M 393216 > $out/${v}_$rep.json 2> $out/${v}_$rep.err || exit 1
  done
done
