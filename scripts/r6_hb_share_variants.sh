# The fused hidden backward's compiled variants (RSLRL_HB_VARIANT "BD,LA") at the 16,384-env share's 98,304-row
# mini-batches (12 tiles per slice), rocprof of the share's bench per variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6hbv}
mkdir -p $o
for v in 1,2 1,4 1,1 2,0 1,3; do
  RSLRL_HB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats_${v/,/_} -o s16k -- python3 bench.py --global-num-envs 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > /dev/null 2>&1
  echo variant $v rc=$?
done
