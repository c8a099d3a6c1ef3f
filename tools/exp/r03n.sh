# Round 3 session N: ordered batches binned like the order-free ones (lists sorted in LDS by the raster):
# fuzz replays (binned default, and NR_ORD_BINNED=0 = the global-sort path), GPU suite, C5 A/B.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_binned.log 2>&1
rc=$?; tail -2 gpurun_out/dbg_binned.log; echo "replay binned rc=$rc"; [ $rc -eq 0 ] || exit $rc
NR_ORD_BINNED=0 timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_sorted.log 2>&1
rc=$?; tail -2 gpurun_out/dbg_sorted.log; echo "replay sorted rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFG=c5 STEPS=20 bash tools/exp/ab_env.sh NR_ORD_BINNED=0 NR_ORD_BINNED=1 NR_ORD_BINNED=0 NR_ORD_BINNED=1 || exit $?
timeout -k 10 200 python bench.py --config c5 --steps 20 --no-cpu-baseline --no-extra > gpurun_out/c5_line.log 2>&1; tail -1 gpurun_out/c5_line.log | cut -c1-300
