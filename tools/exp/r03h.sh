# Round 3 session H: knobs on one rank's 8-way share (host validation, plan kernel, wide instance), C3 timeline.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BENCH_ARGS="--emulate-shards 8 --root-slots equal" bash tools/exp/ab_env.sh "NR_KNOWN_SIZES=1" "NR_KNOWN_SIZES=2" "NR_PLAN_SMALL=1" "NR_KNOWN_SIZES=2,NR_PLAN_SMALL=1" "NR_WIDE_HEAVY=1" "NR_BIN_SETS=2" "NR_KNOWN_SIZES=1" "NR_KNOWN_SIZES=2" "NR_PLAN_SMALL=1" "NR_KNOWN_SIZES=2,NR_PLAN_SMALL=1"
bash tools/exp/tl.sh "c3|" && NR_KNOWN_SIZES=2 bash tools/exp/tl.sh "n8k2|--emulate-shards 8 --root-slots equal"
