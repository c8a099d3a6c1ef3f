# Round 3 session AA: k_vis item classes -- 10 (nb12, HEAD), 14 (nb16) or 18 (nb20) equal bins of the one-slice range:
# fuzz replay and GPU suite with nb16, A/B on C3 and 1M tris at 1080p.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/nb16.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_nb16.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_nb16.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_nb16.log 2>&1; rc=$?; echo "pytest nb16 rc=$rc"; tail -3 gpurun_out/pytest_nb16.log; }
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 nb12 nb16 nb20 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 3 nb12 nb16 nb20 || exit $?
