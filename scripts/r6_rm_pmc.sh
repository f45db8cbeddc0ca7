# SQ counters of the one-launch rollout forward at 65,536 rows (C3's rollout), two passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rmpmc}
mkdir -p $o
P="python3 scripts/rollout_mlp_ab.py --num-envs 65536 --steps 60 --rounds 1 --graph 0 --modes 1 --out $o/ab.json"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $o/sq1 -o run -- $P > $o/sq1.log 2>&1 || { tail -5 $o/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $o/sq2 -o run -- $P > $o/sq2.log 2>&1 || { tail -5 $o/sq2.log; exit 1; }
python3 scripts/kernel_pmc_table.py $o rollout_mlp_kernel 100
