# A/B on one box: act() graph on/off x synthetic env fused/torch, default bench (C3), alternating.
set -e
mkdir -p gpurun_out/rab
for rep in 1 2; do
  for cfg in "1 fused" "0 fused" "1 torch" "0 torch"; do
    set -- $cfg
    RSLRL_ACT_GRAPH=$1 RSLRL_SYNTH_ENV=$2 timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --steps 15 > gpurun_out/rab/g$1_$2_$rep.json 2>/dev/null
  done
done
