# Builds the library of a git revision (default HEAD) into tools/exp/<name>.so for A/B runs against the
# working tree (tools/exp/ab_var.sh).  Usage: bash tools/exp/build_ref.sh [rev] [name]
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
REV=${1:-HEAD}
NAME=${2:-base}
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" libnativecpurenderer_amd/csrc | tar -x -C "$TMP"
make -C "$ROOT" -j8 SRC="$TMP/libnativecpurenderer_amd/csrc" OBJ="$TMP/obj" LIB="$ROOT/tools/exp/$NAME.so" \
    "$ROOT/tools/exp/$NAME.so" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
rm -rf "$TMP"
echo "built tools/exp/$NAME.so from $REV"
