# Round 3 session U: the shading hash pass entering only the first pixel of each winner's run along a tile row (hr1,
# the working tree) vs every pixel (hr0): fuzz replay, GPU suite, A/B on C3, the 8-way share, C2, 1M tris at 1080p.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 hr0 hr1 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 hr0 hr1 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 hr0 hr1 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 hr0 hr1 || exit $?
