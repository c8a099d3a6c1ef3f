# PMC passes over the binning kernels (k_free_count / plan / emit)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_bin; mkdir -p $OUT; export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --steps 3 --warmup 1"
KR="k_free_count|k_free_plan|k_free_emit"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "$KR" -d $OUT/a -o run --output-format csv -- python3 $B > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$KR" -d $OUT/b -o run --output-format csv -- python3 $B > $OUT/b.log 2>&1 || exit 1
echo ok
