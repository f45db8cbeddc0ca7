# Build rsl_rl_amd/lib/variants/<name>/librslrl_amd.so with mlp_fwd_stream.o from <src.hip> [hipcc flags] (diagnostic / A/B builds, never shipped).
set -e
name=$1; src=$2; shift 2
d=rsl_rl_amd/lib/variants/$name
mkdir -p $d/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 -Iinclude -Irsl_rl_amd/csrc "$@" -c $src -o $d/obj/mlp_fwd_stream.o
objs=$(ls rsl_rl_amd/lib/obj/*.o | grep -v mlp_fwd_stream.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/librslrl_amd.so $objs $d/obj/mlp_fwd_stream.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,librslrl_amd.so
