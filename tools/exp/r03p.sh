# Round 3 profile session: GPU suite, C5 full-unit A/B, C3 kernel trace + PMC passes (tools/profile.sh), per-config traffic JSONs.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p_pytest.log 2>&1 || { tail -30 gpurun_out/r03p_pytest.log; exit 1; }
tail -2 gpurun_out/r03p_pytest.log
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 lm0 lm1 || exit 1
bash tools/exp/ab_env.sh "NR_GRID_DIV=1" "NR_GRID_DIV=2" "NR_GRID_DIV=3" "NR_GRID_DIV=1" "NR_GRID_DIV=2" || exit 1
bash tools/profile.sh c3 r03p || exit 1
python tools/pmc_summary.py gpurun_out/prof_r03p > gpurun_out/prof_r03p/summary.txt; head -12 gpurun_out/prof_r03p/summary.txt
bash tools/pmc_traffic.sh c3 "" && bash tools/pmc_traffic.sh c3_1080p "--config c3_1080p" && bash tools/pmc_traffic.sh c2 "--config c2" && \
bash tools/pmc_traffic.sh c5 "--config c5" && bash tools/pmc_traffic.sh c3_shard0of8 "--emulate-shards 8 --root-slots equal" && \
bash tools/pmc_traffic.sh c3_shard0of4 "--emulate-shards 4 --root-slots equal" && bash tools/pmc_traffic.sh c3_shard0of2 "--emulate-shards 2 --root-slots equal"
