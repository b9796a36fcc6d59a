# round 3: evaluator test, rocprof kernel stats of the bench (profiles/r3), march kernel traces
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_eval.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3e_tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
rm -rf gpurun_out/r3_prof gpurun_out/march_trace
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline > gpurun_out/r3e_bench_under_rocprof.json 2> gpurun_out/r3e_bench.log
r=$?; echo "bench rc=$r"; if [ $r -ne 0 ]; then exit $r; fi
for dt in bf16 fp32; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/march_trace/$dt -o m --output-format csv -- python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9 > gpurun_out/march_trace_$dt.log 2>&1
r=$?; echo "trace $dt rc=$r"; tail -2 gpurun_out/march_trace_$dt.log; if [ $r -ne 0 ]; then exit $r; fi
done
find gpurun_out/r3_prof gpurun_out/march_trace -name "*.csv" | head -20
exit $rc
