# Round 6: compute_returns_slots forms -- GPU tests, then the probe under rocprofv3 (kernel durations, csv)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=${1:-gpurun_out/r6}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gae.py tests/test_gpu_minibatch.py -m gpu > $o/gae_tests.log 2>&1 || { tail -40 $o/gae_tests.log; exit 1; }
tail -3 $o/gae_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/gae_prof -o gae -- python3 scripts/gae_probe.py --reps 40 --n 65536 32768 16384 --forms 0 1 2 3 --coop 0 --out $o/gae_probe.json > $o/gae_probe.log 2>&1
echo probe rc=$?
grep '^{' $o/gae_probe.log | cut -c1-220
