# Round 6 checkpoint: the whole GPU suite, smoke(), the default bench line, rocprof kernel stats of the C3 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6full}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 600 python3 bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_default.json')); print('C3', d['value'], d['ms_per_step'], 'update', d['update_env_steps_per_s'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']); print({k: v['value'] for k, v in d.get('extra_configs', {}).items()}); print('cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
echo stats rc=$?
