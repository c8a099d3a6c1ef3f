set -e
O=gpurun_out/r05au; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default_steps20.json 2> $O/b.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --emulate-shards 8 --no-cpu-baseline --no-extra > $O/bench_n8share_steps20.json 2>> $O/b.err
timeout -k 10 120 python bench.py --config c3_1080p --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_1080p_steps20.json 2>> $O/b.err
for f in $O/*.json; do echo $f; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d['ms_per_step'], d.get('roofline',{}).get('frac'), {k:(v.get('ms_per_step') if isinstance(v,dict) else v) for k,v in d.get('extra',{}).items()} if 'extra' in d else '')" $f; done
