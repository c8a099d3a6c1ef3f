# Round 6: non-temporal vertex loads in the warm binning (k_bin_warm reads every triangle's positions once
# per frame, beside the raster: EXP_NTLD, tools/exp/ntld.so) against the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-ntld1}
for cfg in c3 c3_1080p c2; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $cfg" TAG=$T/$cfg bash tools/gpu_session.sh "abl:default%tools/exp/ntld.so%default%tools/exp/ntld.so" || exit 1
done
STEPS=100 WARM=50 BENCH_ARGS="--emulate-shards 8 --root-slots equal" TAG=$T/n8 bash tools/gpu_session.sh "abl:default%tools/exp/ntld.so%default%tools/exp/ntld.so" || exit 1
