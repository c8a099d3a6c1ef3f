# A/B under the 3-wave k_vis: shading hash slots NR_HTS 1024 / 256 vs 512 (base = HEAD), C3 only (the variants
# change every instance's LDS; C3 runs the 3-wave one).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base hts1k hts256
