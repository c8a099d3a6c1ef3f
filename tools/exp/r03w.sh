# Round 3 session W: the ordered raster's blend-only loop skipping the lane-mask reads for wave blocks a triangle covers
# entirely (full1: a second span-phase ballot marks them) vs reading them for every block (full0 = HEAD): fuzz replay
# and GPU suite with full1, A/B on C5 (20 steps, 3 rounds).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/full1.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_full1.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_full1.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_full1.log 2>&1; rc=$?; echo "pytest full1 rc=$rc"; tail -3 gpurun_out/pytest_full1.log; }
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 full0 full1 || exit $?
