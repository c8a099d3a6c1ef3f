# Round 3 session C: GPU suite (ordered-raster setup records + slot merge), C5 line, split-limit A/B (C3).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03c_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r03c_c5.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r03c_c5.log').read().strip().splitlines()[-1]);print('c5', d['ms_per_step'], d['kernel_us'], d.get('valu_roofline',{}).get('frac'))"
bash tools/exp/ab_env.sh "NR_SPLIT_AT=1024" "NR_SPLIT_AT=640,NR_DSLICE=320" "NR_SPLIT_AT=512,NR_DSLICE=256" "NR_SPLIT_AT=768,NR_DSLICE=384" "NR_SPLIT_AT=1024,NR_DSLICE=512" "NR_SPLIT_AT=1024,NR_DSLICE=256" "NR_SPLIT_AT=512,NR_DSLICE=512" "NR_SPLIT_AT=640,NR_DSLICE=192" "NR_SPLIT_AT=1024" "NR_SPLIT_AT=640,NR_DSLICE=320" "NR_SPLIT_AT=512,NR_DSLICE=256"
