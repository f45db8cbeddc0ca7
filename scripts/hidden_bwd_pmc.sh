# Counters over the fused hidden-layer backward (scripts/hidden_bwd_probe.py --only fused) and, for comparison, the
# separate launches it replaces; summarise with scripts/mlp_pmc_summary.py DIR (kernel x6_hidden_bwd_pair).
set -e
out=${1:-gpurun_out/hbpmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/hidden_bwd_probe.py --M 393216 --iters 6"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- $P --only fused > $out/trace.json 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/sq1 -o run -- $P --only fused > $out/sq1.json 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $out/sq2 -o run -- $P --only fused > $out/sq2.json 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/mlp_$c -o run -- $P --only fused > $out/mlp_$c.json 2>&1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/cal_$c -o run -- ./scripts/pmc_pattern_probe.bin > $out/cal_$c.log 2>&1
done
