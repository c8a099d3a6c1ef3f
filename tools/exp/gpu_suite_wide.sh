# GPU suite by default and with the 512-thread k_vis instance taken whenever a batch has a dense tile
# (NR_WIDE_HEAVY large), so that its 1024-slot hash table is exercised across the suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_w.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_w.log
NR_WIDE_HEAVY=100000000 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_w_force.log 2>&1; echo "pytest forced rc=$?"; tail -1 gpurun_out/pytest_w_force.log
