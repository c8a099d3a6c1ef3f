# Round 3 session E: k_vis per-item timeline (times variant), default split and 1024/512.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_pytest.log 2>&1 || { tail -30 gpurun_out/r03e_pytest.log; exit 1; }
tail -2 gpurun_out/r03e_pytest.log
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
cp tools/exp/times.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 200 python tools/exp/item_times.py c3 > gpurun_out/r03e_items_default.txt 2>&1; rc=$?; cat gpurun_out/r03e_items_default.txt | head -14
[ $rc -eq 0 ] && NR_SPLIT_AT=1024 NR_DSLICE=512 timeout -k 10 200 python tools/exp/item_times.py c3 > gpurun_out/r03e_items_512.txt 2>&1; cat gpurun_out/r03e_items_512.txt | head -14
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
