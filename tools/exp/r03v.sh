# Round 3 session V: the ordered raster's next-chunk setup records and colours copied global -> LDS by wave 0
# (global_load_lds) while the current chunk blends (g1) vs loaded by the setup phase (g0): fuzz replay and GPU suite
# with g1 (the working tree), A/B on C5 and on the blended/ordered GPU tests' shapes (C5 at 20 steps, 3 rounds).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_g1.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_g1.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_g1.log 2>&1; rc=$?; echo "pytest g1 rc=$rc"; tail -3 gpurun_out/pytest_g1.log; }
[ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 g0 g1 || exit $?
