# A/B of variant libraries (tools/exp/<v>.so) in one session, alternating, N reps: ab_var.sh "<bench args>" reps v1 v2 ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
args=$1; reps=$2; shift 2
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
for r in $(seq $reps); do
  for v in "$@"; do
    cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 100 $args > gpurun_out/abv.json 2>&1 || { cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so; exit 1; }
    echo "$v $args $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
  done
done
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
