# SQ counters over the RND probe, two passes, each its own time-limited run.
set -e
out=gpurun_out/rndpmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 scripts/rnd_probe.py 20 > $out/probe.json
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $out/p1 -o run -- python3 scripts/rnd_probe.py 3 > $out/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/p2 -o run -- python3 scripts/rnd_probe.py 3 > $out/p2.log 2>&1
