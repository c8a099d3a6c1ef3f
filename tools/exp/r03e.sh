# Round 3 session E: GPU suite on the working tree, then A/B of HEAD (base) against the list/vertex prefetch
# two chunks ahead (pf2): C3 and one rank's 8-way share.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
bash tools/exp/ab_var.sh "" 3 base pf2 || exit $?
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 base pf2 || exit $?
bash tools/exp/ab_var.sh "--config c2" 2 base pf2
