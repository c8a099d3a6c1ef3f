# Round 3 session L: persistent k_vis with one queue counter (NR_VIS_PERSIST=1): fuzz replay, A/B on C3, 8-way, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
NR_VIS_PERSIST=1 timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_persist.log 2>&1
rc=$?; tail -2 gpurun_out/dbg_persist.log; echo "replay rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
BENCH_ARGS="--emulate-shards 8 --root-slots equal" bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
CFG=c2 bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
