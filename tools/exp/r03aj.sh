# Round 3 session AJ: k_vis slicing knobs re-swept under the linear item classes (C3 and 1M tris at 1080p, 2 rounds):
# slice target 384/512/768, split threshold 768/1024/1536, dense slice 512/1024.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in c3 c3_1080p; do for r in 1 2; do
  CFG=$cfg bash tools/exp/ab_env.sh NR_SLICE_TARGET=512 NR_SLICE_TARGET=384 NR_SLICE_TARGET=768 NR_SPLIT_AT=768 NR_SPLIT_AT=1536 NR_DSLICE=512 || exit $?
done; done
