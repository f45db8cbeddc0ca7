set -e
mkdir -p gpurun_out
timeout -k 10 200 python scripts/h3_probe.py > gpurun_out/h3_probe.json 2> gpurun_out/h3_probe.err
