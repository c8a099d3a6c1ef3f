set -e
mkdir -p gpurun_out/r05ay
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05ay/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ay/smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05ay/bench.json 2> gpurun_out/r05ay/bench.err
tail -n 2 gpurun_out/r05ay/tests.log; tail -n 2 gpurun_out/r05ay/smoke.log; cat gpurun_out/r05ay/bench.json
