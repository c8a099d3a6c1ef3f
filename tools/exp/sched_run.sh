# Item timelines of k_vis (times variant) at N=1 and one 8-way share, and their list-schedule simulations.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
cp tools/exp/times.so libnativecpurenderer_amd/libNativeCPURenderer.so
for sh in 1 8; do
  ITEM_SHARDS=$sh timeout -k 10 200 python tools/exp/item_times.py > gpurun_out/items_n$sh.log 2>&1 || { cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; cat gpurun_out/items_n$sh.log | tail; exit 1; }
  mv gpurun_out/item_times.npy gpurun_out/item_times_n$sh.npy
  cat gpurun_out/items_n$sh.log
  for g in 0 1 2; do python tools/exp/sched_sim.py gpurun_out/item_times_n$sh.npy 1024 $g; done
done
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
