# Round 3 session A: GPU suite, driver-style bench line, then A/B of the Gouraud direct-shading variants.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03a_bench.log 2>&1 || { tail -20 gpurun_out/r03a_bench.log; exit 1; }
tail -c 300 gpurun_out/r03a_bench.log
bash tools/exp/ab_var.sh "--no-extra" 2 base gd1 gd2 gd4
