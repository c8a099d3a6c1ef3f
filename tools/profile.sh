# rocprofv3 runs of bench.py: one kernel-trace --stats pass, then PMC passes
# (each counter group in its own run, kernel-trace only beside --pmc), all
# restricted to the dominant kernel.  Usage: bash tools/profile.sh <config> <tag>
# (PMC=0: the kernel trace only)
cd $GRAFT_REPO_ROOT
CFG=${1:-c3}
TAG=${2:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline --no-extra $BENCH_EXTRA"
run() {  # name, timeout, args...
  local name=$1; shift; local t=$1; shift
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1|2) return 0;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
run list 60 rocprofv3 -L
grep -oE "^[[:space:]]*(SQ_|TCC_|TCP_|GRBM_|FETCH|WRITE)[A-Za-z0-9_]*" $OUT/list.log | sort -u > $OUT/counter_names.txt
run trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH --steps 10 --warmup 2
[ "${PMC:-1}" = 1 ] || { ls -R $OUT | head -20; exit 0; }
KR=${KERNEL_REGEX:-"k_vis|k_resolve|k_tile_raster"}
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_fetch -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_write -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
run pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "$KR" -d $OUT/pmc_sq1 -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
run pmc_sq2 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "$KR" -d $OUT/pmc_sq2 -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
run pmc_sq3 300 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU --kernel-include-regex "$KR" -d $OUT/pmc_sq3 -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
run pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KR" -d $OUT/pmc_tcc -o run --output-format csv -- python3 $BENCH --steps 3 --warmup 1
ls -R $OUT | head -50
