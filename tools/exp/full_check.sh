set -e
mkdir -p gpurun_out/r05at
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05at/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05at/smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05at/bench.json 2> gpurun_out/r05at/bench.err
tail -n 2 gpurun_out/r05at/tests.log; tail -n 2 gpurun_out/r05at/smoke.log; cat gpurun_out/r05at/bench.json
