# Round 3 session H: fuzz replay + GPU suite with 16x16 ordered blocks (ord16 = working tree), A/B of f32 spans in
# the 3-wave k_vis (s32w3 vs pf2 = HEAD) and of the ordered raster's block width on C5, shading / item clocks of HEAD.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_ord16.log 2>&1
rc=$?; tail -3 gpurun_out/dbg_ord16.log; echo "replay rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "--config c5 --steps 20" 2 ord64 ord32 ord16 || exit $?
bash tools/exp/ab_var.sh "" 3 pf2 s32w3 || exit $?
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
for v in sht times; do
  cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so
  if [ $v = sht ]; then timeout -k 10 120 python tools/exp/shade_times.py; else timeout -k 10 120 python tools/exp/item_times.py; fi
  rc=$?; cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
done
