# Round 6: the C3 frame with YUV420P frame output measured slower than with u8 RGB output (0.1305 vs
# 0.1239 ms in the r06fin2 default line): same-process-order-free A/B of the two outputs, and YUV420P
# with non-temporal byte stores (tools/exp/ntyuv.so, EXP_NT_YUV).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=${TAG:-yuv1}; O=gpurun_out/$T; mkdir -p $O
for cfg in c3 c3_1080p; do
  for rep in 1 2; do
    for v in "yuv|--frame-output yuv420p" "rgb|--frame-output rgb" "ntyuv|--frame-output yuv420p --lib tools/exp/ntyuv.so"; do
      n=${v%%|*}; a=${v#*|}
      echo "== $cfg $n $rep" | tee -a $O/session.txt
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 100 --warmup 50 --config $cfg $a > $O/${cfg}_${n}_$rep.log 2>&1 || exit 1
      tail -1 $O/${cfg}_${n}_$rep.log | cut -c1-200 | tee -a $O/session.txt
    done
  done
done
