set -e
out=gpurun_out/r4/diag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in default nostore noio bfirst0; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 120 python scripts/gemm_ab.py --variants default --rounds 3 --M 393216 > $out/gemm_$v.json 2>/dev/null
  RSLRL_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/sq1_$v -o run -- python3 scripts/mlp_pair_probe.py --iters 6 > $out/sq1_$v.json 2>&1
done
