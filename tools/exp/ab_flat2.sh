export TAG=${TAG:-flat3}
bash tools/gpu_session.sh test || exit 1
if grep -q "failed\|illegal\|rror" gpurun_out/$TAG/01_test.log; then echo "GPU suite not green: no A/B"; exit 1; fi
NR_LIB=tools/exp/probe.so timeout -k 10 120 python tools/exp/probe_items.py c2 > gpurun_out/$TAG/probe_c2.txt 2>&1 || exit 1
for c in ${CONFIGS:-c2 c3}; do
  STEPS=100 WARM=50 BENCH_ARGS="--config $c" TAG=$TAG/$c bash tools/gpu_session.sh abl:default%tools/exp/base.so || exit 1
done
