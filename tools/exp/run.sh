# A/B kernel variants: each tools/exp/<v>.so swapped in for the library, one bench line each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
for v in "$@"; do
  if [ "$v" = base ]; then cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; else cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so; fi
  if [ "$v" = sht ]; then timeout -k 10 120 python tools/exp/shade_times.py; continue; fi
  if [ "$v" = plant ]; then timeout -k 10 120 python tools/exp/plan_times.py; continue; fi
  if [ "$v" = times ]; then
    timeout -k 10 300 python tools/exp/item_times.py $ITEM_CFG > gpurun_out/exp_$v.log 2>&1; rc=$?; cat gpurun_out/exp_$v.log | tail -12
    [ $rc -eq 0 ] || break; continue
  fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/exp_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_$v.log) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/exp_$v.log)"
  [ $rc -eq 0 ] || break
done
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
