# A/B: 64x16 tiles (NR_TH=16 build, tools/exp/th16.so) vs 64x32 (base); then the GPU suite under th16 (sharding helpers assume 32-row bands).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base th16 && bash tools/exp/ab_var.sh "--emulate-shards 8" 2 base th16 && bash tools/exp/ab_var.sh "--emulate-shards 4" 2 base th16 && bash tools/exp/ab_var.sh "--config c2" 2 base th16 && bash tools/exp/ab_var.sh "--config c5 --steps 20" 1 base th16
cp tools/exp/th16.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 > gpurun_out/pytest_th16.log 2>&1
tail -15 gpurun_out/pytest_th16.log
cp tools/exp/base.so libnativecpurenderer_amd/libNativeCPURenderer.so
