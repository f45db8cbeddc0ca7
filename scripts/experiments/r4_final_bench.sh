# round-4 final bench lines: the default command (CPU baseline + extra configs) and the strong-scaling shares
set -e
o=gpurun_out/r4f2
mkdir -p $o
timeout -k 10 600 python bench.py > $o/bench_default.json 2> $o/bench_default.err
tail -c 600 $o/bench_default.json
timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k.json 2> $o/b16k.err
timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline > $o/b16k_2.json 2> $o/b16k_2.err
timeout -k 10 240 python bench.py --global-num-envs 32768 --no-extra --no-cpu-baseline --steps 10 > $o/b32k.json 2> $o/b32k.err
python - <<'P'
import json
for f in ("b16k", "b16k_2", "b32k"):
    d = json.loads(open(f"gpurun_out/r4f2/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("phases_last_iter"))
P
