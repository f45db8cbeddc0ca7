# Round 6 closing numbers on one box: the GPU suite, smoke(), the default bench line (C3 + extras + CPU baseline), the
# strong-scaling shares (16,384 / 32,768 envs) and C4's 131,072 envs on one GPU, rocprof kernel stats of the C3 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6final}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 600 python3 bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
for n in 16384 32768 131072; do
  timeout -k 10 400 python3 bench.py --global-num-envs $n --no-cpu-baseline --no-extra > $o/b$n.json 2> $o/b$n.err || { tail -20 $o/b$n.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/bench_stats.json 2> $o/bench_stats.err
echo stats rc=$?
python3 - <<PY
import json
d = json.load(open("$o/bench_default.json"))
print("C3", d["value"], d["ms_per_step"], "update", d["update_env_steps_per_s"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["traffic"])
print({k: v["value"] for k, v in d.get("extra_configs", {}).items()}, "cpu", d["cpu_baseline"]["value"])
for n in (16384, 32768, 131072):
    b = json.load(open(f"$o/b{n}.json"))
    print(n, b["value"], b["ms_per_step"], b["update_env_steps_per_s"], b["roofline"]["kernel"], b["roofline"]["frac"], b["roofline"]["traffic"])
PY
