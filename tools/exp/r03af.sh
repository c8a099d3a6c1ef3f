# Round 3 session AF: ordered batches beside the previous ordered raster planned by a 512-thread k_free_plan_r
# (NR_ORD_PLAN512=1, the working tree) vs the 1024-thread one (0): fuzz replay, GPU suite, A/B on C5 (20 steps).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFG=c5 STEPS=20 bash tools/exp/ab_env.sh NR_ORD_PLAN512=0 NR_ORD_PLAN512=1 NR_ORD_PLAN512=0 NR_ORD_PLAN512=1 NR_ORD_PLAN512=0 NR_ORD_PLAN512=1 || exit $?
