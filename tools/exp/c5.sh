cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c5}; do
timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/$c.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/$c.log').read().strip().splitlines()[-1]);print('$c', d['ms_per_step'],d['kernel_us'])"
done
