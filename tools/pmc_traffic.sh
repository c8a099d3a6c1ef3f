# HBM traffic of the dominant kernel for one bench configuration: two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE: separate runs, no trace domains), then tools/pmc_json.py writes gpurun_out/pmc_<tag>.json
# (copy it to profiles/ to have bench.py report it as roofline.traffic for that configuration and share).
# Usage: bash tools/pmc_traffic.sh <tag> "<bench args>"   e.g. c3_shard0of8 "--emulate-shards 8 --root-slots equal"
# The passes bin inline (NR_WARM_INLINE=1): --pmc serialises dispatches, so a raster waiting on the same-queue token
# of a binning beside it (k_gate_wait) would wait out its 1 s timeout and run the all-triangle fallback.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=$1; ARGS=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmct_$TAG
mkdir -p $OUT
KR=${KERNEL_REGEX:-"k_vis|k_tile_raster"}
for c in FETCH_SIZE WRITE_SIZE; do
  NR_WARM_INLINE=1 timeout -k 10 240 rocprofv3 --pmc $c --kernel-include-regex "$KR" -d $OUT/$c -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-extra --steps 3 --warmup 1 --clock-settle-ms 0 $ARGS > $OUT/$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -5 $OUT/$c.log; exit 1; }
done
python tools/pmc_json.py $OUT $TAG "$ARGS"
