# A/B of runtime knobs: each argument is an env assignment list ("A=1,B=2"), one bench line each.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-extra $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['roofline']['kernel_us'])"
done
