# Round 3 session T: emit compaction for sharded frames (count appends the triangles touching owned rows, emit walks
# only those) and the blend-only loop's per-triangle data by lane reads (rl1) vs LDS reads (rl0): fuzz replay (main,
# rl1), GPU suite, A/B NR_COMPACT=0/1 on the emulated 8-, 4- and 2-way shares, rl0/rl1 on C5; k_vis issuing its first
# item, list and depth loads together (early) vs one after another (late) on C3, the 8-way share, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 8 4 2; do
  BENCH_ARGS="--emulate-shards $s --root-slots equal" bash tools/exp/ab_env.sh NR_COMPACT=0 NR_COMPACT=1 NR_COMPACT=0 NR_COMPACT=1 || exit $?
done
bash tools/exp/ab_var.sh "" 3 late early || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 late early || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 late early || exit $?
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/rl1.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_rl1.log 2>&1
rc=$?; cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; echo "rl1 fuzz"; tail -2 gpurun_out/fuzz_rl1.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 rl0 rl1 || exit $?
