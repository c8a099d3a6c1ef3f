set -e
O=gpurun_out/r05as; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_warm_gpu.py tests/test_fast_clear_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra >> $O/pre_1080.jsonl
  timeout -k 10 120 python bench.py --lib tools/exp/nosum.so --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra >> $O/nosum_1080.jsonl
  timeout -k 10 120 python bench.py --config c3 --steps 100 --warmup 20 --emulate-shards 8 --no-cpu-baseline --no-extra >> $O/pre_8w.jsonl
  timeout -k 10 120 python bench.py --lib tools/exp/nosum.so --config c3 --steps 100 --warmup 20 --emulate-shards 8 --no-cpu-baseline --no-extra >> $O/nosum_8w.jsonl
done
tail -n 2 $O/tests.log
for f in $O/*.jsonl; do echo $f; python -c "import json,sys; print([round(json.loads(l)['ms_per_step'],4) for l in open(sys.argv[1])])" $f; done
