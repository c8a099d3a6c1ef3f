# Round 3 session K: GPU suite (working tree, per-item grid), persistent k_vis over the work queue
# (NR_VIS_PERSIST=1): fuzz replay (parity), then A/B vs the per-item grid on C3, the 8-way share and C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
NR_VIS_PERSIST=1 timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_persist.log 2>&1
rc=$?; tail -3 gpurun_out/dbg_persist.log; echo "replay rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
BENCH_ARGS="--emulate-shards 8 --root-slots equal" bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
CFG=c2 bash tools/exp/ab_env.sh NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 NR_VIS_PERSIST=0 NR_VIS_PERSIST=1 || exit $?
