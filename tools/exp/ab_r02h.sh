cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
for a in "" "--emulate-shards 8" "--emulate-shards 4" "--config c2"; do
  for pr in 1 0; do
    NR_PLAN_REG=$pr timeout -k 10 120 python bench.py --no-cpu-baseline --no-kernel-timing --steps 200 $a > gpurun_out/ab.json 2>&1 || exit 1
    echo "planreg=$pr $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
  done
done
done
