# Round 6: the degree-5 ELU polynomial -- the whole GPU suite on the new build, then alternating bench A/B against the
# previous build (rsl_rl_amd/lib/variants/elu9: the degree-9 Taylor form) and the streaming-forward probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6elu}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
B=rsl_rl_amd/lib/variants/elu9/librslrl_amd.so
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/bench_new$rep.json 2>/dev/null || exit 1
  RSLRL_AMD_LIB=$B timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/bench_old$rep.json 2>/dev/null || exit 1
done
python3 - <<PY
import json
for k in ("new", "old"):
    v = [json.load(open(f"$o/bench_{k}{r}.json"))["value"] for r in (1, 2, 3)]
    print(k, [round(x / 1e6, 3) for x in v])
PY
