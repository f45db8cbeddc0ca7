set -e
o=gpurun_out/gap
mkdir -p $o
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/bench1.json 2> $o/bench1.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr -o run -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-extra > $o/bench_tr.json 2> $o/bench_tr.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/bench2.json 2> $o/bench2.err
