# N>1 bench orchestration on ONE GPU (gloo, no RCCL gather): calibration, barriers, max-over-ranks timing, JSON
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
N=${N:-2}
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 20 --warmup 3 --gloo-test $BENCH_ARGS > gpurun_out/bench_multi_$N.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/bench_multi_$N.log | tail -1 | head -c 1500; echo; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_multi_$N.log
exit $rc
