# time every variants/*.so with the MLP microbench, then the default build's GPU tests
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
: > gpurun_out/variants.json
for v in variants/*.so; do
  n=$(basename $v .so)
  for M in 786432 262144; do
    timeout -k 10 120 python tools/mlp_bench.py --lib $v --M $M > gpurun_out/v.json 2>>gpurun_out/variants.err || exit 1
    echo "$n $(cat gpurun_out/v.json)" >> gpurun_out/variants.json
  done
done
cat gpurun_out/variants.json
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log
exit $rc
