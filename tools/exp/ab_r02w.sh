# A/B: hash slots of the 3-wave k_vis instance, 2048 (h2k) vs 1024 (base = HEAD), C3 and 1M triangles at 1080p;
# then the GPU suite at HEAD, by default and with the 3-wave instance forced on every batch.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base h2k && bash tools/exp/ab_var.sh "--config c3_1080p" 2 base h2k || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_hts.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_hts.log
NR_VIS_WPE3=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_hts_force.log 2>&1; echo "pytest forced rc=$?"; tail -1 gpurun_out/pytest_hts_force.log
