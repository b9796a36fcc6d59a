export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
echo rc=$rc
tail -3 gpurun_out/gputests.log
tail -1 gpurun_out/smoke.log
tail -3 gpurun_out/bench.log
exit $rc
