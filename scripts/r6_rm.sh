# One-launch rollout forward (rollout_mlp.hip): parity tests, then same-box A/B of the bench at the N = 8 share and C3
# (RSLRL_ROLLOUT_MLP=0 = the layer-by-layer launches), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rm}
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout_mlp.py tests/test_gpu_pair.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for r in 1 2; do
  for v in 0 1; do
    RSLRL_ROLLOUT_MLP=$v timeout -k 10 300 python3 bench.py --global-num-envs 16384 --no-cpu-baseline --no-extra > $o/b16k_rm${v}_$r.json 2> $o/b16k_rm${v}_$r.err || { tail -20 $o/b16k_rm${v}_$r.err; exit 1; }
    RSLRL_ROLLOUT_MLP=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $o/c3_rm${v}_$r.json 2> $o/c3_rm${v}_$r.err || { tail -20 $o/c3_rm${v}_$r.err; exit 1; }
    python3 - <<PY
import json, statistics
for n in ("b16k", "c3"):
    d = json.load(open("$o/" + n + "_rm${v}_$r.json"))
    print(n, "rm=$v", "round $r", d["value"], d["ms_per_step"], "collection ms", statistics.median(d["phases_timed_ms"]["collection"]), "learn ms", statistics.median(d["phases_timed_ms"]["learn"]))
PY
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats16k -o b16k -- python3 bench.py --global-num-envs 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/stats16k.json 2> $o/stats16k.err
echo stats rc=$?
