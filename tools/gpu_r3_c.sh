# round 3 (re-entry): the whole -m gpu suite on the current head, smoke(), then the default bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread \
  > gpurun_out/r3c_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r3c_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3c_smoke.log 2>&1
r=$?; tail -2 gpurun_out/r3c_smoke.log; if [ $r -ne 0 ]; then exit $r; fi
timeout -k 10 500 python3 -u bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.log
r=$?; echo "bench rc=$r"; tail -c 600 gpurun_out/r3c_bench.json
if [ $r -ne 0 ]; then exit $r; fi
exit $rc
