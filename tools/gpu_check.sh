# One GPU session: parity tests, then (if no crash) the debug probe and a bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
if [ -n "$GPU_DEBUG" ]; then timeout -k 10 300 python $GPU_DEBUG > gpurun_out/debug.log 2>&1; echo "debug rc=$?"; tail -20 gpurun_out/debug.log; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 $BENCH_ARGS > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -3 gpurun_out/bench.log
