# Round 3 close-out profile: the default bench line (N=1, C3, cpu_baseline + extra lines), the kernel trace + PMC
# passes of C3 and of C5 (SQ issue counters of the ordered raster), and the HBM traffic JSONs of C3 and C5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_default.err; exit 1; }
tail -c 600 gpurun_out/bench_default.json
bash tools/profile.sh c3 r03z_c3 || exit $?
KERNEL_REGEX="k_tile_raster" bash tools/profile.sh c5 r03z_c5 || exit $?
bash tools/pmc_traffic.sh c3 "" || exit $?
KERNEL_REGEX="k_tile_raster" bash tools/pmc_traffic.sh c5 "--config c5" || exit $?
