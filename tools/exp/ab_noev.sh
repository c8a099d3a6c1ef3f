# Round 6 probe (timing only): the ~4.7 us gap after every k_vis -- is it the raster's completion event
# (hipExtLaunchKernel stop event F.evVis)?  tools/exp/noev.so launches an inline warm batch's k_vis
# without it (EXP_NOVISEV; the set's reuse is stream-ordered when inline).  1080p (inline binning).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-noev1}
TAG=$T/tr bash tools/gpu_session.sh "ktrace:--steps,20,--warmup,5,--config,c3_1080p,--lib,tools/exp/noev.so" || exit $?
STEPS=100 WARM=50 BENCH_ARGS="--config c3_1080p" TAG=$T/c3_1080p bash tools/gpu_session.sh "abl:default%tools/exp/noev.so" || exit 1
