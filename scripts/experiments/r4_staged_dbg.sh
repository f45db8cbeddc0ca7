set -e
out=gpurun_out/r4/staged
rm -rf $out; mkdir -p $out /tmp/sd
timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/a.pt --M 2048 > $out/det_a.txt
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/unstaged/librslrl_amd.so timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/b.pt --M 2048 > $out/det_b.txt
timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/a2.pt --M 2048 > $out/det_a2.txt
timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/big.pt --M 98304 > $out/det_big.txt
python scripts/gemm_dump.py --cmp /tmp/sd/a.pt /tmp/sd/a2.pt > $out/cmp_aa.txt 2>&1 || true
python scripts/gemm_dump.py --cmp /tmp/sd/a.pt /tmp/sd/b.pt > $out/cmp.txt 2>&1 || true
rm -rf /tmp/sd
