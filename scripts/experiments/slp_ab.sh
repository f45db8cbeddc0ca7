# A/B of diagnostic builds (rsl_rl_amd/lib/variants/<v>/librslrl_amd.so): the streaming forward with a cheaper / no ELU
# epilogue, and whole libraries without the compiler's packed-f32 (SLP) vectorisation -- per-kernel probes, alternating
# processes on one box, then the bench under the default and the no-SLP library.
set -e
o=${1:-gpurun_out/slp}
mkdir -p $o
lib() { if [ $1 = main ]; then echo rsl_rl_amd/lib/librslrl_amd.so; else echo rsl_rl_amd/lib/variants/$1/librslrl_amd.so; fi; }
for rep in 1 2; do
  for v in main expelu noelu noslp noslpall; do
    RSLRL_AMD_LIB=$(lib $v) timeout -k 10 120 python3 scripts/fwd_stream_probe.py > $o/fs_${v}_$rep.json
  done
  for v in main noslpall; do
    RSLRL_AMD_LIB=$(lib $v) timeout -k 10 120 python3 -u scripts/hidden_bwd_probe.py --M 393216 > $o/hb_${v}_$rep.json 2> $o/hb_${v}_$rep.err
    RSLRL_AMD_LIB=$(lib $v) timeout -k 10 120 python3 -u scripts/actor_head_probe.py --M 393216 > $o/ah_${v}_$rep.json 2> $o/ah_${v}_$rep.err
  done
done
for rep in 1 2; do
  for v in main noslpall; do
    RSLRL_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err
  done
done
