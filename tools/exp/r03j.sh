# Round 3 session J/M: GPU suite at the working tree, the default bench line (with extras),
# then the C3 profile (kernel trace + PMC passes) and the per-config HBM traffic of C3 and C5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh c3 r03q || exit $?
bash tools/pmc_traffic.sh c3 "" || exit $?
bash tools/pmc_traffic.sh c5 "--config c5" || exit $?
