set -e
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 120 python scripts/x6_probe.py
done
