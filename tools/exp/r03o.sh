# Round 3 session O: binned ordered batches with the per-tile list sort on the binning stream (k_tile_sort):
# fuzz replay, GPU suite, C5 A/B vs the global-sort path.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_binned.log 2>&1
rc=$?; tail -2 gpurun_out/dbg_binned.log; echo "replay binned rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFG=c5 STEPS=20 bash tools/exp/ab_env.sh NR_ORD_BINNED=0 NR_ORD_BINNED=1 NR_ORD_BINNED=0 NR_ORD_BINNED=1 || exit $?
timeout -k 10 200 python bench.py --config c5 --steps 20 --no-cpu-baseline --no-extra > gpurun_out/c5_line.log 2>&1; tail -1 gpurun_out/c5_line.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernel_us'])"
