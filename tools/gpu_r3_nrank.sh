# round 3: the N > 1 bench path rehearsed on one GPU (gloo; the driver's 8-GPU runs use RCCL):
# N = 2 and 4 ranks sharing cuda:0, the default workload (3 dtypes, renders, march, bake), few steps
export TMPDIR=/tmp NERF_BENCH_BACKEND=gloo
cd $GRAFT_REPO_ROOT
for N in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) \
    bench.py --gpus $N --steps 3 --warmup 1 > gpurun_out/bench_n${N}_gloo.json 2> gpurun_out/bench_n${N}_gloo.err
  r=$?; echo "N=$N rc=$r"; tail -c 300 gpurun_out/bench_n${N}_gloo.json; echo
  if [ $r -ne 0 ]; then tail -20 gpurun_out/bench_n${N}_gloo.err; exit $r; fi
done
