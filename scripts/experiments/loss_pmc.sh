# SQ counters over the loss microbench (depth 1 and 2, 256 blocks); one pass per counter set.
set -e
mkdir -p gpurun_out/losspmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 1 2; do
RSLRL_LOSS_DEPTH=$d timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/losspmc/d$d -o run -- python3 scripts/hotpath_microbench.py --only loss --iters 50 > gpurun_out/losspmc/d$d.log 2>&1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/losspmc/stats -o run -- python3 scripts/hotpath_microbench.py --only loss --iters 200 > gpurun_out/losspmc/stats.log 2>&1
