set -e
O=gpurun_out/r05ao; mkdir -p $O
for r in 1 2; do
  for d in r4 bis/7dd915f bis/ce5cf4c bis/3699a65 bis/834a3cb bis/8960898 bis/6a06c69 cur; do
    n=$(echo $d | tr '/' '_')
    if [ $d = cur ]; then
      timeout -k 10 120 python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra >> $O/$n.jsonl
    else
      (cd tools/exp/$d && timeout -k 10 120 python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra) >> $O/$n.jsonl
    fi
  done
done
for f in $O/*.jsonl; do echo $f; python -c "import json,sys; print([round(json.loads(l)['ms_per_step'],4) for l in open(sys.argv[1])])" $f; done
