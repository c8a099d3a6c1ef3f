# Round 3 session AI: k_vis shading pass storing each fully shaded tile row as packed words staged in LDS (pk1 = the
# working tree: 16-byte f64 rgb words and 4-byte u8 words, contiguous across lanes) vs per-pixel strided stores (pk0):
# fuzz replay, GPU suite, A/B on C3, 1M tris at 1080p, the 8-way share, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 pk0 pk1 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 pk0 pk1 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 pk0 pk1 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 pk0 pk1 || exit $?
