# Build rsl_rl_amd/lib/variants/<name>/librslrl_amd.so: the in-tree objects with gae.o rebuilt with [extra hipcc flags]
# (e.g. -DRSLRL_GAE_STAMPS for scripts/gae_stamps.py; never shipped).  Run `make -C rsl_rl_amd/csrc` first.
set -e
name=$1; shift
d=rsl_rl_amd/lib/variants/$name
mkdir -p $d/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 -Iinclude -Irsl_rl_amd/csrc "$@" -c rsl_rl_amd/csrc/gae.hip -o $d/obj/gae.o
objs=$(ls rsl_rl_amd/lib/obj/*.o | grep -v "/gae.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/librslrl_amd.so $objs $d/obj/gae.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,librslrl_amd.so
