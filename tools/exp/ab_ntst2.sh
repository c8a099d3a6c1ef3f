# Round 6: non-temporal raster output stores as the shipped default (out_store; the ordered raster's
# write-back too) against the previous build (tools/exp/base.so): GPU suite, then three interleaved
# pairs per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-ntst2}
TAG=$T bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$T/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
for cfg in c3 c3_1080p c2 c5; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $cfg" TAG=$T/$cfg bash tools/gpu_session.sh "abl:default%tools/exp/base.so%default%tools/exp/base.so%default%tools/exp/base.so" || exit 1
done
STEPS=100 WARM=50 BENCH_ARGS="--emulate-shards 8 --root-slots equal" TAG=$T/n8 bash tools/gpu_session.sh "abl:default%tools/exp/base.so%default%tools/exp/base.so" || exit 1
