# Round 3 session S: emit compaction for sharded frames (count appends the triangles touching owned rows, emit walks
# only those): fuzz replay, GPU suite, A/B NR_COMPACT=0/1 on the emulated 8-, 4- and 2-way shares.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -3 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 8 4 2; do
  BENCH_ARGS="--emulate-shards $s --root-slots equal" bash tools/exp/ab_env.sh NR_COMPACT=0 NR_COMPACT=1 NR_COMPACT=0 NR_COMPACT=1 || exit $?
done
