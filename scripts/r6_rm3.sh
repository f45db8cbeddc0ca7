# one-launch rollout forward: kernel stats of both forms (rollout step only), kernel traces of the 16,384-env bench, bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6rm3}
mkdir -p $o
for v in 0 1; do
  RSLRL_ROLLOUT_MLP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s$v -o s -- python3 scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 100 --rounds 1 --graph 0 --out $o/ab_prof$v.json > $o/prof$v.log 2>&1 || { tail -20 $o/prof$v.log; exit 1; }
done
for v in 0 1; do
  RSLRL_ROLLOUT_MLP=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/t$v -o t -- python3 bench.py --global-num-envs 16384 --steps 4 --warmup 2 --no-cpu-baseline --no-extra > $o/t$v.json 2> $o/t$v.err || { tail -20 $o/t$v.err; exit 1; }
done
echo traced
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
