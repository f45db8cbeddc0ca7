# strong-scaling share (16384 envs): per-iteration host phase times over repeated runs (collection-time variance)
set -e
o=gpurun_out/r4/share_diag
mkdir -p $o
for rep in 1 2 3; do
  timeout -k 10 240 python bench.py --global-num-envs 16384 --no-extra --no-cpu-baseline --steps 15 > $o/b16k_$rep.json 2> $o/b16k_$rep.err
  python -c "
import json; d=json.loads(open('$o/b16k_$rep.json').read().strip().splitlines()[-1])
print($rep, d['value'], d['ms_per_step'], d['phases_timed_ms'])"
done
