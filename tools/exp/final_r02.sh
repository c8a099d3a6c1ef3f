# Round-2 close-out on one box: C3 kernel trace + PMC passes (tools/profile.sh), then the bench line
# repeated at the driver's shape (20 steps, 5 warmup) and at 100 steps, plus C2 / C5 lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/profile.sh c3 r02f || exit $?
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/bench_lines.txt 2>/dev/null || exit $?
  timeout -k 10 180 python bench.py --steps 100 --warmup 10 --no-cpu-baseline >> gpurun_out/bench_lines.txt 2>/dev/null || exit $?
done
timeout -k 10 180 python bench.py --config c2 --steps 100 --no-cpu-baseline >> gpurun_out/bench_lines.txt 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 20 --no-cpu-baseline >> gpurun_out/bench_lines.txt 2>/dev/null || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_lines.txt
