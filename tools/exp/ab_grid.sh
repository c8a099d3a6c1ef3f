# A/B: k_vis grid from known / last item counts (NR_GRID_EST=1, default) vs the capacity bound (0)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_grid_tests.log 2>&1 || { tail -30 gpurun_out/r02_grid_tests.log; exit 1; }
tail -1 gpurun_out/r02_grid_tests.log
for r in 1 2; do
  bash tools/exp/ab_env.sh NR_GRID_EST=0 NR_GRID_EST=1 || exit 1
  BENCH_ARGS="--emulate-shards 8" bash tools/exp/ab_env.sh NR_GRID_EST=0 NR_GRID_EST=1 || exit 1
  BENCH_ARGS="--emulate-shards 4" bash tools/exp/ab_env.sh NR_GRID_EST=0 NR_GRID_EST=1 || exit 1
  CFG=c2 bash tools/exp/ab_env.sh NR_GRID_EST=0 NR_GRID_EST=1 || exit 1
done
