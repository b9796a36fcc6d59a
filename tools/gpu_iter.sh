# one GPU iteration: MLP microbench, GPU parity tests, full bench (each step time-limited)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/mlp_bench.py > gpurun_out/mlpb.json 2>gpurun_out/mlpb.err && \
timeout -k 10 120 python tools/mlp_bench.py --M 262144 >> gpurun_out/mlpb.json 2>>gpurun_out/mlpb.err && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
echo rc=$rc
cat gpurun_out/mlpb.json
tail -5 gpurun_out/gputests.log
tail -1 gpurun_out/bench.log
exit $rc
