# Round 3 session I: GPU suite with 32x8 ordered blocks (working tree = ord32), fuzz replays of the tagged plan
# totals (nowb) and of the keys-first shading pass (kf), A/B ord32 (HEAD) / nowb / kf on C3, the 8-way share, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
for v in nowb kf; do
  cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so
  timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_$v.log 2>&1
  rc=$?; cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; tail -3 gpurun_out/dbg_$v.log; echo "replay $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/exp/ab_var.sh "" 3 ord32 nowb kf || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 3 ord32 nowb kf || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 ord32 nowb kf || exit $?
