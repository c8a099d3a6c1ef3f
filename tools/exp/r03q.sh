# Round 3 session Q: device-side binning -> raster hand-off (NR_GATE=1): GPU suite with it, A/B vs the cross-queue
# event wait on C3, the emulated 8-way share, C2 and C5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
NR_GATE=1 timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest (gate) rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_env.sh NR_GATE=0 NR_GATE=1 NR_GATE=0 NR_GATE=1 NR_GATE=0 NR_GATE=1 || exit $?
BENCH_ARGS="--emulate-shards 8 --root-slots equal" bash tools/exp/ab_env.sh NR_GATE=0 NR_GATE=1 NR_GATE=0 NR_GATE=1 || exit $?
CFG=c2 bash tools/exp/ab_env.sh NR_GATE=0 NR_GATE=1 NR_GATE=0 NR_GATE=1 || exit $?
CFG=c5 STEPS=20 bash tools/exp/ab_env.sh NR_GATE=0 NR_GATE=1 || exit $?
