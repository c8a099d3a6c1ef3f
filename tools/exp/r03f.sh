# Round 3 session F: GPU suite on the working tree (shading slot reuse), A/B of pf2 (HEAD) / slot / f32 spans in the
# 3-wave instance (s32w3, slot32), then shading phase clocks (sht) and per-item clocks (times) of pf2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 pf2 slot s32w3 slot32 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 pf2 slot slot32 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 pf2 slot slot32 || exit $?
bash tools/exp/ab_var.sh "--config c5 --steps 20" 2 ord64 ord32 ord16 || exit $?
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
for v in sht times; do
  cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so
  if [ $v = sht ]; then timeout -k 10 120 python tools/exp/shade_times.py; else timeout -k 10 120 python tools/exp/item_times.py; fi
  rc=$?; cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
done
