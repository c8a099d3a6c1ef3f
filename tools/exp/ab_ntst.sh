# Round 6: the ~4.7 us gap after every k_vis (kernel trace, r06fin2/tr) -- the end-of-kernel release
# writing back the L2s' dirty lines? Non-temporal stores for every raster output (tools/exp/ntst.so,
# EXP_NTST: out_store = __builtin_nontemporal_store) against the shipped build: kernel traces + bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-ntst1}
TAG=$T/tr bash tools/gpu_session.sh "ktrace:--steps,20,--warmup,5,--config,c3_1080p" "ktrace:--steps,20,--warmup,5,--config,c3_1080p,--lib,tools/exp/ntst.so" || exit $?
for cfg in c3 c3_1080p c2; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $cfg" TAG=$T/$cfg bash tools/gpu_session.sh "abl:default%tools/exp/ntst.so" || exit 1
done
STEPS=100 WARM=50 BENCH_ARGS="--emulate-shards 8 --root-slots equal" TAG=$T/n8 bash tools/gpu_session.sh "abl:default%tools/exp/ntst.so" || exit 1
