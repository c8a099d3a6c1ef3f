cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c3 c2}; do BENCH_ARGS="--config $c" bash tools/exp/run.sh base old $EXTRA || exit 1; done
