# Round 3 session D: split-limit A/B with the batched slot reduction (C3, and one rank's 8-way share).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/exp/ab_env.sh "NR_SPLIT_AT=1024" "NR_SPLIT_AT=1024,NR_DSLICE=512" "NR_SPLIT_AT=768,NR_DSLICE=384" "NR_SPLIT_AT=640,NR_DSLICE=320" "NR_SPLIT_AT=1024" "NR_SPLIT_AT=1024,NR_DSLICE=512" "NR_SPLIT_AT=768,NR_DSLICE=384"
BENCH_ARGS="--emulate-shards 8 --root-slots equal" bash tools/exp/ab_env.sh "NR_SPLIT_AT=1024" "NR_SPLIT_AT=1024,NR_DSLICE=256" "NR_SPLIT_AT=512,NR_DSLICE=256" "NR_SPLIT_AT=256,NR_DSLICE=128" "NR_SPLIT_AT=1024"
CFG=c5 STEPS=20 bash tools/exp/ab_var.sh "--config c5 --steps 20" 3 bp0 bp1
