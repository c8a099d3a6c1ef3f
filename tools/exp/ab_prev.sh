set -e
O=gpurun_out/r05ax; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_warm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for r in 1 2 3; do
  for v in cur prev; do
    L=""; [ $v = prev ] && L="--lib tools/exp/prev.so"
    true
    timeout -k 10 120 python bench.py $L --steps 100 --warmup 20 --emulate-shards 8 --no-cpu-baseline --no-extra >> $O/${v}_8w.jsonl
    timeout -k 10 120 python bench.py $L --config c3_1080p --steps 100 --warmup 20 --no-cpu-baseline --no-extra >> $O/${v}_1080.jsonl
  done
done
for f in $O/*.jsonl; do echo $f; python -c "import json,sys; print([round(json.loads(l)['ms_per_step'],4) for l in open(sys.argv[1])])" $f; done
