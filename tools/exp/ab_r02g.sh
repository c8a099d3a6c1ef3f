cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
for a in "" "--emulate-shards 8" "--emulate-shards 4" "--emulate-shards 2"; do
  for kp in "1 0" "1 1" "0 0" "0 1"; do
    set -- $kp
    NR_KNOWN_SIZES=$1 NR_STREAM_PRIO=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-kernel-timing --steps 200 $a > gpurun_out/ab.json 2>&1 || exit 1
    echo "known=$1 prio=$2 $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
  done
done
done
