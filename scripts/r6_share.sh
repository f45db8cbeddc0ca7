# Round 6: the N = 8 share (16,384 envs) -- a bench line and a kernel trace of a short run (collection vs GPU idle)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6share}
mkdir -p $o
timeout -k 10 300 python3 bench.py --global-num-envs 16384 --no-cpu-baseline --no-extra > $o/b16k.json 2> $o/b16k.err || { tail -20 $o/b16k.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/b16k.json')); print(d['value'], d['ms_per_step'], d['update_env_steps_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o b16k -- python3 bench.py --global-num-envs 16384 --steps 4 --warmup 2 --no-cpu-baseline --no-extra > $o/b16k_trace.json 2> $o/b16k_trace.err
echo trace rc=$?
