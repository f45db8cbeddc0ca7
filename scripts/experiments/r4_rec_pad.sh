# rollout_record occupancy experiment: dynamic-LDS padding limits the resident blocks per CU (pad32768: ~4,
# pad54000: 2, pad100000: 1), so that later blocks' loads overlap earlier blocks' stores
set -e
o=gpurun_out/r4/rec_pad
mkdir -p $o
for rep in 1 2 3; do
for v in default pad32768 pad54000 pad100000; do
  if [ $v = default ]; then L=rsl_rl_amd/lib/librslrl_amd.so; else L=rsl_rl_amd/lib/variants/$v/librslrl_amd.so; fi
  RSLRL_AMD_LIB=$L timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 6 --warmup 2 > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err
  python -c "
import json; d=json.loads(open('$o/c3_${v}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v', $rep, d['value'], r['kernel'], r['mean_launch_us'], r['frac'], r['call_span_us'])"
done
done
