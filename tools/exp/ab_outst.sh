# Round 6: does the ~4.7 us gap after every k_vis come from the end-of-kernel L2 write-back?  Raster
# outputs stored write-through (relaxed atomic stores: agent scope = sc1, tools/exp/sta.so; system scope =
# sc0 sc1, tools/exp/sts.so) against the shipped non-temporal stores: kernel traces and bench pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-outst1}
TAG=$T/tr bash tools/gpu_session.sh "ktrace:--steps,20,--warmup,5,--config,c3_1080p,--lib,tools/exp/sta.so" "ktrace:--steps,20,--warmup,5,--config,c3_1080p,--lib,tools/exp/sts.so" || exit $?
for cfg in c3 c3_1080p; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $cfg" TAG=$T/$cfg bash tools/gpu_session.sh "abl:default%tools/exp/sta.so%tools/exp/sts.so" || exit 1
done
STEPS=100 WARM=50 BENCH_ARGS="--emulate-shards 8 --root-slots equal" TAG=$T/n8 bash tools/gpu_session.sh "abl:default%tools/exp/sta.so%tools/exp/sts.so" || exit 1
