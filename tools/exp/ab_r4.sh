set -e
O=gpurun_out/r05an; mkdir -p $O
for r in 1 2 3; do
  for fo in rgb yuv420p; do
    timeout -k 10 120 python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output $fo --no-cpu-baseline --no-extra >> $O/cur_1080_$fo.jsonl
    (cd tools/exp/r4 && timeout -k 10 120 python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output $fo --no-cpu-baseline --no-extra) >> $O/r4_1080_$fo.jsonl
  done
  timeout -k 10 120 python bench.py --config c2 --steps 100 --warmup 200 --no-cpu-baseline --no-extra >> $O/cur_c2.jsonl
  (cd tools/exp/r4 && timeout -k 10 120 python bench.py --config c2 --steps 100 --warmup 200 --frame-output yuv420p --no-cpu-baseline --no-extra) >> $O/r4_c2.jsonl
done
for f in $O/*.jsonl; do echo $f; python -c "import json,sys; print([round(json.loads(l)['ms_per_step'],4) for l in open(sys.argv[1])])" $f; done
