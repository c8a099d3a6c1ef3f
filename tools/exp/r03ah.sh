# Round 3 session AH: a sharded frame's plan beside the previous raster by a 512-thread k_free_plan_r
# (NR_SHARD_PLAN512=1, the working tree) vs the 1024-thread one (0): fuzz replay, GPU suite (its sharded cases run the
# 512-thread plan), A/B on the emulated 8-, 4- and 2-way shares.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 8 4 2; do
  BENCH_ARGS="--emulate-shards $s --root-slots equal" bash tools/exp/ab_env.sh NR_SHARD_PLAN512=0 NR_SHARD_PLAN512=1 NR_SHARD_PLAN512=0 NR_SHARD_PLAN512=1 NR_SHARD_PLAN512=0 NR_SHARD_PLAN512=1 || exit $?
done
