set -e
mkdir -p gpurun_out/r05al
for r in 1 2 3; do
  for v in 1 0; do
    NR_COLD_GATE=$v timeout -k 10 120 python bench.py --config c3_animated --steps 50 --warmup 10 >> gpurun_out/r05al/anim_cg$v.jsonl
    NR_COLD_GATE=$v timeout -k 10 120 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05al/c3_cg$v.jsonl
  done
done
for f in gpurun_out/r05al/*.jsonl; do echo $f; python -c "import json,sys; print([round(json.loads(l)['ms_per_step'],4) for l in open(sys.argv[1])])" $f; done
