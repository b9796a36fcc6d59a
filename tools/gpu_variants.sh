# time every variants/*.so in interleaved rounds (one process) for each MLP dtype given in
# $VAR_DTYPES (default fp32), then the default build's GPU tests
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
libs=$(ls variants/*.so | paste -sd, -)
: > gpurun_out/variants.json
for dt in ${VAR_DTYPES:-fp32}; do
  timeout -k 10 300 python tools/mlp_bench.py --dtype $dt --libs $libs --M 524288 --reps 5 --rounds 5 >> gpurun_out/variants.json 2>>gpurun_out/variants.err || exit $?
done
cat gpurun_out/variants.json; tail -3 gpurun_out/variants.err
[ -n "$VAR_NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log
exit $rc
