# A/B under the 3-wave k_vis with its 1024-slot hash table (base = HEAD): probe limit 8 / 32 (mp8, mp32) vs 16, and
# 333 staged records (rec: NR_REC_EXTRA=26000, LDS ~50 KB) vs 280, C3 (the variants change every instance).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_var.sh "" 3 base mp8 mp32 rec
