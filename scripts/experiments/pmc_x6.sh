# SQ counter passes over the GEMM probe (one PROBE_ONLY direction): wave-state breakdown, instruction
# mix, memory-pipe pressure.  Usage: PROBE_ONLY=fwd bash scripts/pmc_x6.sh <outdir>
set -e
out=${1:-gpurun_out/pmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv --pmc "$@" -d $out/p$pass -o run -- python3 scripts/mlp_kernel_probe.py > $out/p$pass.json
}
pass=1 run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC
pass=2 run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM
pass=3 run GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
