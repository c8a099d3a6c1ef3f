# A/B of the flattened chunk raster (shipped build) against tools/exp/base.so;
# the bench lines only after a green GPU suite
export TAG=${TAG:-flat}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
for c in ${CONFIGS:-c3 c2 c3_1080p}; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $c" TAG=$TAG/$c bash tools/gpu_session.sh abl:default%tools/exp/base.so || exit 1
done
