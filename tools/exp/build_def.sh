# Builds tools/exp/<name>.so with one source file compiled with extra defines (the other objects from build/obj).
# Usage: bash tools/exp/build_def.sh <name> <source basename, e.g. nr_tri_ordered> -DX=1 ...
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
NAME=$1; SRCB=$2; shift 2
SRC=$ROOT/libnativecpurenderer_amd/csrc
OBJS=$(ls $ROOT/build/obj/*.o | grep -v "/$SRCB.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc -Wno-pass-failed "$@" \
    -I$SRC -c $SRC/$SRCB.hip -o /tmp/_def_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/exp/$NAME.so $OBJS /tmp/_def_$NAME.o -ldl
echo "built tools/exp/$NAME.so"
