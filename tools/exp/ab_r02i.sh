cd $GRAFT_REPO_ROOT
bash tools/exp/ab_var.sh "" 3 head q0 q1 q2 && bash tools/exp/ab_var.sh "--emulate-shards 8" 3 head q0 q1 q2
