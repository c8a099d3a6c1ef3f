# Round 3 session AB: k_vis reading per-triangle setup records that k_free_count formed (vrec1: screen vertices, edge
# slopes, 1/den, z0 and depth differences, 112 B per triangle) vs setting each triangle up from its vertices in every
# tile (nb12 = HEAD): fuzz replay and GPU suite with vrec1, A/B on C3, 1M tris at 1080p, the 8-way share, C2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so; cp tools/exp/vrec1.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python tools/debug_fuzz.py tools/exp/fuzz_examples.pkl > gpurun_out/fuzz_vrec1.log 2>&1
rc=$?; tail -2 gpurun_out/fuzz_vrec1.log
[ $rc -eq 0 ] && { timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_vrec1.log 2>&1; rc=$?; echo "pytest vrec1 rc=$rc"; tail -3 gpurun_out/pytest_vrec1.log; }
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; [ $rc -eq 0 ] || exit $rc
bash tools/exp/ab_var.sh "" 3 nb12 vrec1 || exit $?
bash tools/exp/ab_var.sh "--config c3_1080p" 2 nb12 vrec1 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 nb12 vrec1 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 nb12 vrec1 || exit $?
