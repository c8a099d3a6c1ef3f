# Round 6: barrier-free block raster for the ordered path (k_block_raster) against the tile raster
# (NR_ORD_RASTER=0), with and without the culled queue, 4 or 3 waves per SIMD (tools/exp/wpe3.so).
export TAG=${TAG:-blk1}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
STEPS=50 BENCH_ARGS="--config c5" TAG=$TAG/c5 bash tools/gpu_session.sh "ab:NR_ORD_RASTER=0%NR_ORD_RASTER=1%NR_ORD_RASTER=2" || exit 1
STEPS=50 WARM=10 BENCH_ARGS="--config c5" TAG=$TAG/c5w bash tools/gpu_session.sh "abl:default%tools/exp/wpe3.so" || exit 1
