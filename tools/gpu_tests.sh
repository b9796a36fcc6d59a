# the GPU test suite alone (time-limited), log under gpurun_out/
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log
exit $rc
