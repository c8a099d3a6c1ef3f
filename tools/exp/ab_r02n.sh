# A/B: k_vis compiled for 3 waves/SIMD (NR_VIS_WAVES_PER_EU=3: up to 168 VGPRs, no spills) vs 4 (base = HEAD).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base w3 && bash tools/exp/ab_var.sh "--emulate-shards 8" 2 base w3 && bash tools/exp/ab_var.sh "--config c2" 2 base w3
