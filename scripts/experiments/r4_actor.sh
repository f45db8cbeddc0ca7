#!/bin/bash
# round 4: the fused actor head -- parity tests, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r4/actor
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_actor_head.py \
    > gpurun_out/r4/actor/tests.log 2>&1 || { tail -40 gpurun_out/r4/actor/tests.log; exit 1; }
tail -3 gpurun_out/r4/actor/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_value_head.py \
    tests/test_gpu_update.py tests/test_gpu_update_variants.py > gpurun_out/r4/actor/tests2.log 2>&1 \
    || { tail -40 gpurun_out/r4/actor/tests2.log; exit 1; }
tail -3 gpurun_out/r4/actor/tests2.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-extra > gpurun_out/r4/actor/bench.json 2> gpurun_out/r4/actor/bench.err \
    || { tail -20 gpurun_out/r4/actor/bench.err; exit 1; }
python - <<'P'
import json
d = json.loads(open("gpurun_out/r4/actor/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d["roofline"])[:300])
for k, v in sorted(d["mlp_kernels"].items(), key=lambda kv: -kv[1]["ms_per_step"]):
    print(f'{k:60s} {v["mean_us"]:9.2f} {v["ms_per_step"]:8.3f}')
print(json.dumps(d["hot_path"]["kernels"].get("ppo_loss")))
P
