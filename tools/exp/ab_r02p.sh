# A/B: 3-wave k_vis with 378 staged shading records (rx: NR_REC_EXTRA=32256, 53.5 KB LDS, still 3 workgroups/CU)
# vs 280 (base = HEAD 30f4da7), C3 and 1M triangles at 1080p.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base rx && bash tools/exp/ab_var.sh "--config c3_1080p" 2 base rx
