# run one python script against a variant library: run1.sh <variant> <script> [args]
cd $GRAFT_REPO_ROOT
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
cp tools/exp/$1.so libnativecpurenderer_amd/libNativeCPURenderer.so
shift
timeout -k 10 200 python "$@"; rc=$?
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
exit $rc
