# Round 3 session R: empty tiles folded into the largest single-slice k_vis items (fold = working tree) vs one item per
# empty tile (nofold): GPU suite, fuzz replay, A/B on C3, the 8-way share, C2, 1M tris at 1080p; item clocks.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 nofold fold || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 nofold fold || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 nofold fold || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 nofold fold || exit $?
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/times.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 120 python tools/exp/item_times.py; rc=$?; cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; exit $rc
