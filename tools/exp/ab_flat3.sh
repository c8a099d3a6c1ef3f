export TAG=${TAG:-flat4}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
NR_LIB=tools/exp/probe.so timeout -k 10 120 python tools/exp/probe_items.py c2 > gpurun_out/$TAG/probe_c2.txt 2>&1 || exit 1
for c in ${CONFIGS:-c2}; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $c" TAG=$TAG/$c bash tools/gpu_session.sh abl:default%${OTHER:-tools/exp/flat1.so} || exit 1
done
timeout -k 10 120 python tools/exp/host_cost.py > gpurun_out/$TAG/host_cost_1.txt 2>&1 || exit 1
timeout -k 10 120 python tools/exp/host_cost.py 8 > gpurun_out/$TAG/host_cost_8.txt 2>&1 || exit 1
