set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05ap; mkdir -p $O
cd $R/tools/exp/r4 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/r4 -o run --output-format csv -- python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra > $O/r4.json
cd $R/tools/exp/bis/7dd915f && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/b7 -o run --output-format csv -- python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra > $O/b7.json
cd $R && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/cur -o run --output-format csv -- python bench.py --config c3_1080p --steps 100 --warmup 200 --frame-output rgb --no-cpu-baseline --no-extra > $O/cur.json
for d in r4 b7 cur; do echo == $d; f=$(find $O/$d -name "*kernel_stats.csv" | head -1); python -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:6]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2))
" $f; done
