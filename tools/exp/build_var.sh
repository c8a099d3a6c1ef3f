# Variant library: one source file rebuilt with extra defines, linked with the other objects.
# Usage: bash tools/exp/build_var.sh <name> <source basename, e.g. nr_tri_ordered> "-DX=1 -DY=2"  -> tools/exp/<name>.so
set -e
cd "$(dirname "$0")/../.."
name=$1; src=$2; defs=$3
objs=$(ls build/obj/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc -Wno-pass-failed $defs \
  -Ilibnativecpurenderer_amd/csrc -c libnativecpurenderer_amd/csrc/$src.hip -o /tmp/_var_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/exp/$name.so $objs /tmp/_var_$name.o -ldl
