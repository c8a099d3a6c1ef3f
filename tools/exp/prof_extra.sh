# Round-end evidence: kernel-trace stats of an emulated 8-way shard (one rank's frame) and the C2/C5 bench lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof_r01d; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01d/n8 -o run --output-format csv -- python3 bench.py --emulate-shards 8 --no-cpu-baseline --steps 30 --warmup 3 > gpurun_out/prof_r01d/n8_bench.log 2>&1 || exit $?
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/prof_r01d/bench_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --emulate-shards 2 --no-cpu-baseline --steps 50 > gpurun_out/prof_r01d/emu2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --emulate-shards 4 --no-cpu-baseline --steps 50 > gpurun_out/prof_r01d/emu4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --emulate-shards 8 --no-cpu-baseline --steps 50 > gpurun_out/prof_r01d/emu8.log 2>&1 || exit $?
ls -R gpurun_out/prof_r01d | head
