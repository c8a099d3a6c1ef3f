# Round 6: C5 blend-only loop skipping the step masks of triangles that cover a wave's whole block
# (FULLW) against the round-6 tile raster (tools/exp/base.so).
export TAG=${TAG:-fullw}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
STEPS=50 WARM=10 BENCH_ARGS="--config c5" TAG=$TAG/c5 bash tools/gpu_session.sh "abl:default%tools/exp/base.so" || exit 1
