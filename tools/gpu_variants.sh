# time every variants/*.so in interleaved rounds (one process), then the default build's GPU tests
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
libs=$(ls variants/*.so | paste -sd, -)
timeout -k 10 300 python tools/mlp_bench.py --libs $libs --M 786432 --reps 5 --rounds 5 > gpurun_out/variants.json 2>gpurun_out/variants.err && \
timeout -k 10 300 python tools/mlp_bench.py --libs $libs --M 262144 --reps 5 --rounds 5 >> gpurun_out/variants.json 2>>gpurun_out/variants.err
rc=$?
cat gpurun_out/variants.json; tail -3 gpurun_out/variants.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log
exit $rc
