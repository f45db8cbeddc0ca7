# round-4 closing check after the rollout_record store / log-prob changes: whole GPU suite + smoke, the default bench
# line, the 16384-env share, and the headline command's rocprofv3 kernel stats
set -e
o=gpurun_out/r4e3
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 600 python bench.py > $o/bench_default.json 2> $o/bench_default.err
tail -c 300 $o/bench_default.json
timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k.json 2> $o/b16k.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
python - <<'P'
import json
for f in ("bench_default", "b16k", "bench_stats"):
    d = json.loads(open(f"gpurun_out/r4e3/{f}.json").read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f, d["value"], d["ms_per_step"], r.get("kernel"), r.get("mean_launch_us"), r.get("frac"))
P
