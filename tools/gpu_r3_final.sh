# round 3, final: the whole -m gpu suite, smoke(), the default bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/final_tests.log | tail -3; grep -E "FAILED" gpurun_out/final_tests.log | head -10
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
r=$?; tail -2 gpurun_out/final_smoke.log; if [ $r -ne 0 ]; then exit $r; fi
timeout -k 10 500 python3 -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
r=$?; echo "bench rc=$r"; tail -c 300 gpurun_out/final_bench.json; if [ $r -ne 0 ]; then exit $r; fi
exit $rc
