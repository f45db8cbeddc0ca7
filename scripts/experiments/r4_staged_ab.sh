set -e
out=gpurun_out/r4/staged3
rm -rf $out; mkdir -p $out /tmp/sd
timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/a.pt --M 98304 > $out/det_a.txt
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/unstaged/librslrl_amd.so timeout -k 10 120 python scripts/gemm_dump.py /tmp/sd/b.pt --M 98304 > $out/det_b.txt
python scripts/gemm_dump.py --cmp /tmp/sd/a.pt /tmp/sd/b.pt > $out/cmp.txt 2>&1 || { rm -rf /tmp/sd; cat $out/cmp.txt; exit 3; }
rm -rf /tmp/sd
GV=base,w4 bash scripts/lib_ab.sh rsl_rl_amd/lib/variants/unstaged/librslrl_amd.so $out
