# Register / scratch / occupancy of every kernel instance of one source file
# (-Rpass-analysis=kernel-resource-usage).  Usage: bash tools/kres.sh <file.hip> [name-regex]  (EXTRA: -D flags)
f=$1; re=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-rdc -I$(dirname $f) $EXTRA -c $f -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 "$(dirname "$0")/kres_parse.py" "$re"
