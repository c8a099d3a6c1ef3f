cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/emu
for n in 1 2 4 8; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --emulate-shards $n > gpurun_out/emu/emu$n.json 2>/dev/null || exit 1
  echo "shards=$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/emu/emu$n.json) $(grep -o '"kernel_us": [0-9.]*' gpurun_out/emu/emu$n.json | head -1)"
done
