# Round 3 final line: smoke(), the default bench line of the final tree, its C3 kernel trace, and the kernel traces of
# frames flushed one by one (tools/exp/bench_sync.py: no binning beside the raster) for C3 and C5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_final.err; exit 1; }
tail -c 400 gpurun_out/bench_final.json
PMC=0 bash tools/profile.sh c3 r03zb_c3 || exit $?
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sync_$c -o run --output-format csv -- python3 tools/exp/bench_sync.py $c 30 > gpurun_out/sync_$c.log 2>&1 || { echo "sync $c rc=$?"; tail -5 gpurun_out/sync_$c.log; exit 1; }
  tail -2 gpurun_out/sync_$c.log
done
