# Round 3 session AC = sessions AA + AB in one call (tools/exp/r03aa.sh, tools/exp/r03ab.sh).
cd $GRAFT_REPO_ROOT
bash tools/exp/r03aa.sh || exit $?
bash tools/exp/r03ab.sh
