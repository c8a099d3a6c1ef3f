# Bench lines of the round's final code: C3 (driver shape and 100 steps), C2, C5, C3 at 1080p, emulated 2/4/8-way
# C3 shares, and frames flushed one by one (tools/exp/bench_sync.py).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; O=gpurun_out/final_lines.txt; : > $O
for a in "--steps 20 --warmup 5" "--steps 100" "--config c2 --steps 100" "--config c5 --steps 20" "--config c3_1080p --steps 100" "--emulate-shards 2 --steps 100" "--emulate-shards 4 --steps 100" "--emulate-shards 8 --steps 100"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline $a >> $O 2>/dev/null || exit 1
done
for c in c3 c2; do timeout -k 10 120 python tools/exp/bench_sync.py $c 60 >> $O 2>/dev/null || exit 1; done
grep -o '"ms_per_step": [0-9.]*\|synced.*' $O
