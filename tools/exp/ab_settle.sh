# Round 6: the driver-flag line (20 steps after 5) of C3 reads 4-6 % slower than the same frames later in the
# same process (extra.c3_rgb) or in 100-step runs.  Clock settle 60 ms (shipped) against 250 / 1000 ms of
# untimed frames before the warmup, interleaved, three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-settle1}; O=gpurun_out/$T; mkdir -p $O
for rep in 1 2 3; do
  for s in 60 250 1000; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 --clock-settle-ms $s > $O/c3_s${s}_$rep.log 2>&1 || exit 1
    echo "settle $s rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $O/c3_s${s}_$rep.log)" | tee -a $O/session.txt
  done
done
for rep in 1 2; do
  for s in 60 1000; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 --clock-settle-ms $s --config c3_1080p > $O/p1080_s${s}_$rep.log 2>&1 || exit 1
    echo "1080p settle $s rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $O/p1080_s${s}_$rep.log)" | tee -a $O/session.txt
  done
done
