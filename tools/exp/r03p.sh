# Round 3 session P: GPU suite + fuzz replay with f32 spans in the ordered raster (os32 = working tree), C5 A/B of
# os64 (f64 spans) / os32 / ow6 (6 waves per SIMD, spills).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/dbg_os32.log 2>&1
rc=$?; tail -2 gpurun_out/dbg_os32.log; echo "replay rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 os64 os32 ow6 || exit $?
