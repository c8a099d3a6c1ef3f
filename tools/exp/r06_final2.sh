# The round-6 measurement session (tools/exp/r06_final.sh) plus kernel traces of the C2 and 1080p frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${1:-r06fin2}
bash tools/exp/r06_final.sh "$T" || exit $?
TAG=$T/tr bash tools/gpu_session.sh "ktrace:--steps,20,--warmup,5,--config,c2" "ktrace:--steps,20,--warmup,5,--config,c3_1080p" || exit $?
