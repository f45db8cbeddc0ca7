set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=gpurun_out/r6adam; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_update.py tests/test_gpu_update_c3.py tests/test_gpu_update_variants.py -m gpu > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $o/b.json 2> $o/b.err
python3 -c "
import csv
for r in csv.DictReader(open('$o/stats/c3_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('grad_sq','adam_kernel','fold_batch','gae_fused')): print(r['Name'][:60], float(r['AverageNs'])/1e3)
"
