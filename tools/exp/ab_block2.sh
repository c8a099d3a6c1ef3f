# Round 6: block raster with the software-pipelined cull loop against the tile raster (NR_ORD_RASTER=0).
export TAG=${TAG:-blk2}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
STEPS=50 BENCH_ARGS="--config c5" TAG=$TAG/c5 bash tools/gpu_session.sh "ab:NR_ORD_RASTER=0%NR_ORD_RASTER=2" || exit 1
