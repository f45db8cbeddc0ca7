# Kernel stats of the 16,384-env share's bench (the N = 8 strong-scaling share) on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6share}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o s16k -- python3 bench.py --global-num-envs 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
echo stats rc=$?
