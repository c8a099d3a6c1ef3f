# A/B: shading hash slots of the 512-thread k_vis instance (emulated 4- and 8-way C3 shares run it), 1024 / 2048
# (hw1k, hw2k) vs 512 (base = HEAD).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "--emulate-shards 8" 3 base hw1k hw2k && bash tools/exp/ab_var.sh "--emulate-shards 4" 3 base hw1k hw2k
