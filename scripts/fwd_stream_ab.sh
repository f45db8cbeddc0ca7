# A/B of the square hidden-layer forward pair: streaming kernel (default) vs the tiled one (RSLRL_FWD_STREAM=0),
# alternating processes on one box, then the streaming kernel's SQ counters (clock, MFMA pipe) in their own passes.
set -e
o=${1:-gpurun_out/fsab}
mkdir -p $o
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/fwd_stream_probe.py > $o/stream_$rep.json
  RSLRL_FWD_STREAM=0 timeout -k 10 120 python3 scripts/fwd_stream_probe.py > $o/tiled_$rep.json
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $o/sq1 -o run -- python3 scripts/fwd_stream_probe.py 6 > $o/sq1.json 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $o/sq2 -o run -- python3 scripts/fwd_stream_probe.py 6 > $o/sq2.json 2>&1
