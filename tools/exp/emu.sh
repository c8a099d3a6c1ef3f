# Per-rank frame time of a tile-row shard emulated on one GPU (no gather):
# bash tools/exp/emu.sh "<shard counts>" "<NR_SLICE_TARGET values>"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for t in ${2:-2048}; do
for n in ${1:-1 2 4 8}; do
NR_SLICE_TARGET=$t timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --emulate-shards $n $BENCH_ARGS > gpurun_out/emu_${t}_$n.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/emu_${t}_$n.log').read().strip().splitlines()[-1]);print('target $t shards $n', d['ms_per_step'],d['kernel_us'],d['roofline']['kernel_us'])"
done; done
