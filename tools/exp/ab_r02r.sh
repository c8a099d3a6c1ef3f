# A/B under the 3-wave k_vis (base = HEAD): two directly loaded shading records in flight per thread (ovf2,
# NR_OVF_Q=2; the 3-wave instance has register room) and no raised priority for dense items (hp0, NR_HEAVY_PRIO=0).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base ovf2 hp0
