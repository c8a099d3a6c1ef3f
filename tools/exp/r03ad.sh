# Round 3 session AD: k_vis setup records as planes (vrec2: plane j of triangle t at [j n + t], each chunk load
# contiguous across lanes) vs none (nb12 = HEAD): fuzz replay and GPU suite with vrec2, A/B on C3, 1M tris at 1080p,
# the 8-way share, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/vrec2.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_vrec2.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_vrec2.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_vrec2.log 2>&1; rc=$?; echo "pytest vrec2 rc=$rc"; tail -3 gpurun_out/pytest_vrec2.log; }
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 nb12 vrec2 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 nb12 vrec2 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 nb12 vrec2 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 nb12 vrec2 || exit $?
