# A/B of idle-inline binning on frames synced one by one (tools/exp/bench_sync.py): NR_BIN_IDLE_INLINE=0 vs 1.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2; do for cfg in c3 c2; do for v in 0 1; do
  echo "inline=$v $cfg $(NR_BIN_IDLE_INLINE=$v timeout -k 10 120 python tools/exp/bench_sync.py $cfg 60 2>/dev/null)" || exit 1
done; done; done
