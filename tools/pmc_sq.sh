# SQ issue/stall counters of the dominant kernel for one bench configuration (one --pmc pass, <= 8 SQ counters,
# no trace domains).  SQ_* cycle counters count quad-cycles (MI355X_MICROARCH.md).  Bins inline (NR_WARM_INLINE=1,
# see pmc_traffic.sh).  Usage: bash tools/pmc_sq.sh <tag> "<bench args>"  -> gpurun_out/pmcsq_<tag>/
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=$1; ARGS=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcsq_$TAG
mkdir -p $OUT
KR=${KERNEL_REGEX:-"k_vis|k_tile_raster"}
NR_WARM_INLINE=1 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-include-regex "$KR" -d $OUT -o run \
  --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --steps 3 --warmup 1 --clock-settle-ms 0 $ARGS \
  > $OUT/run.log 2>&1 || { echo "pmc rc=$?"; tail -5 $OUT/run.log; exit 1; }
echo "pmc_sq $TAG done"
