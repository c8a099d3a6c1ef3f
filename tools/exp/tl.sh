# kernel-trace timelines: one rocprofv3 run per bench configuration given as "tag|args"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/tl; export TMPDIR=/tmp
for spec in "$@"; do
  tag=${spec%%|*}; args=${spec#*|}
  timeout -k 10 200 rocprofv3 --kernel-trace $TLFLAGS -d gpurun_out/tl/$tag -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --no-kernel-timing --steps 20 --warmup 3 $args > gpurun_out/tl/$tag.log 2>&1 || exit $?
  f=$(find gpurun_out/tl/$tag -name "*kernel_trace.csv" | head -1)
  python tools/timeline.py $f 3 > gpurun_out/tl/$tag.txt 2>&1
  echo "== $tag"; tail -40 gpurun_out/tl/$tag.txt
done
