# Kernel + memory-copy trace of the 16,384-env share's bench: where the update's permutation upload sits
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6copy}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/trace -o s16k -- python3 bench.py --global-num-envs 16384 --steps 4 --warmup 2 --no-cpu-baseline --no-extra > $o/bench.json 2> $o/bench.err
echo trace rc=$?
