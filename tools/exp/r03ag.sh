# Round 3 session AG: the rasters' output stores (framebuffer, depth, frame output) non-temporal (nt1) vs plain (nt0 =
# the working tree): fuzz replay and GPU suite with nt1, A/B on C3, 1M tris at 1080p, the 8-way share, C2, C5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/nt1.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_nt1.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_nt1.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_nt1.log 2>&1; rc=$?; echo "pytest nt1 rc=$rc"; tail -3 gpurun_out/pytest_nt1.log; }
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 nt0 nt1 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 nt0 nt1 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 nt0 nt1 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 nt0 nt1 || exit $?
bash tools/exp/ab_var.sh "--config c5 --steps 20" 2 nt0 nt1 || exit $?
