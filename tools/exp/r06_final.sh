# Round-6 measurement session: GPU suite, smoke, the driver's bench line, its rocprofv3 kernel stats (C3 and the
# moving-scene line), emulated 2/4/8-way share lines, and the PMC HBM-traffic summaries bench.py reports
# (profiles/pmc_<tag>.json).  Usage (gpurun): bash tools/exp/r06_final.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${1:-r06fin}
TAG=$T bash tools/gpu_session.sh test smoke "bench:--steps,20,--warmup,5" "stats:--steps,20,--warmup,5" \
  "stats:--steps,20,--warmup,5,--config,c3_animated" \
  "bench:--steps,20,--warmup,5,--no-extra,--no-cpu-baseline,--emulate-shards,8,--root-slots,equal" \
  "bench:--steps,20,--warmup,5,--no-extra,--no-cpu-baseline,--emulate-shards,4,--root-slots,equal" \
  "bench:--steps,20,--warmup,5,--no-extra,--no-cpu-baseline,--emulate-shards,2,--root-slots,equal" \
  "bench:--steps,20,--warmup,5,--no-extra,--no-cpu-baseline,--emulate-shards,8,--root-slots,equal,--deliver,bands" || exit $?
for a in "c3_yuv420p|" "c3_animated_yuv420p|--config c3_animated" "c3_1080p_yuv420p|--config c3_1080p" \
         "c2_yuv420p|--config c2" "c5_yuv420p|--config c5" "c3_shard0of8_yuv420p|--emulate-shards 8 --root-slots equal"; do
  bash tools/pmc_traffic.sh "${a%%|*}" "${a#*|}" || exit $?
done
for d in gpurun_out/$T/stats*; do python3 tools/trace_steady.py $d/run_kernel_trace.csv 40 > $d/steady.txt; done
