# Build rsl_rl_amd/lib/variants/<name>/librslrl_amd.so: the in-tree objects with <src>.o rebuilt from
# rsl_rl_amd/csrc/<src>.hip with [extra hipcc flags] (A/B of one kernel file; never shipped).  `make` first.
set -e
name=$1; src=$2; shift 2
d=rsl_rl_amd/lib/variants/$name
mkdir -p $d/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 -Iinclude -Irsl_rl_amd/csrc "$@" -c rsl_rl_amd/csrc/$src.hip -o $d/obj/$src.o
objs=$(ls rsl_rl_amd/lib/obj/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/librslrl_amd.so $objs $d/obj/$src.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,librslrl_amd.so
