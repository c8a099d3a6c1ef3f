mkdir -p gpurun_out/pv
for v in "" 1 2 3 4 5; do
  for c in c2 c3; do
    NR_LIB=tools/exp/probe$v.so timeout -k 10 120 python tools/exp/probe_items.py $c > gpurun_out/pv/probe${v}_$c.txt 2>&1 || exit 1
  done
done
