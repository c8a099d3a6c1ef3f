# Round 3 session F: GPU suite on the current build; A/B: k_vis f32 spans (sp0/sp1), record batching (rq1/rq2), ordered f32 spans (os0/os1, C5); C5 phase clocks; timelines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03f_pytest.log 2>&1 || { tail -30 gpurun_out/r03f_pytest.log; exit 1; }
tail -2 gpurun_out/r03f_pytest.log
bash tools/exp/ab_var.sh "" 3 sp0 sp1 rq1 rq2 || exit 1
bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 os0 os1 || exit 1
bash tools/exp/ab_var.sh "--config c2" 2 sp0 rq2 && bash tools/exp/ab_var.sh "--emulate-shards 8 --root-slots equal" 2 sp0 rq2
cp libnativecpurenderer_amd/libNativeCPURenderer.so /tmp/keep.so
cp tools/exp/oph.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 120 python tools/exp/ordered_phases.py run c5
cp /tmp/keep.so libnativecpurenderer_amd/libNativeCPURenderer.so
bash tools/exp/tl.sh "c3|" "n8|--emulate-shards 8 --root-slots equal"
