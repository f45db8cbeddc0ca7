# Loss kernel with / without an MFMA-heavy GEMM before each launch: event spans, then rocprof kernel stats.
set -e
mkdir -p gpurun_out/lic
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "none" "bf16" "bf16 --gv-pad"; do
  timeout -k 10 120 python scripts/loss_incontext.py --heat $cfg
done
i=0
for cfg in "none" "bf16" "bf16 --gv-pad"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lic/c$i -o run -- python3 scripts/loss_incontext.py --heat $cfg > gpurun_out/lic/c$i.log 2>&1
done
