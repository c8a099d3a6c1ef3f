# Round 3 session I: GPU suite (owned-row histograms), A/B: s0q2 (f64 spans) / s1q2 (f32 spans) / hc (f32 spans + owned-row histograms) on C3, C2, 8-way, 4-way.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03i_pytest.log 2>&1 || { tail -30 gpurun_out/r03i_pytest.log; exit 1; }
tail -2 gpurun_out/r03i_pytest.log
bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 3 s0q2 s1q2 hc || exit 1
bash tools/exp/ab_var.sh "--emulate-shards 4 --root-slots equal" 2 s0q2 s1q2 hc || exit 1
bash tools/exp/ab_var.sh "--config c2" 2 s0q2 s1q2 hc || exit 1
bash tools/exp/ab_var.sh "" 2 s0q2 s1q2 hc
