# round 3: device-count march (persistent MLP, macro-block skip) tests, sweep, trace
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trained.py tests/test_gpu_render.py -m gpu -v -s \
  --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3b_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for dt in bf16 fp32; do
  timeout -k 10 300 python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9,12x2_klow4_t0.9,12x2_klow2_t0.9,16x2_klow4_t0.9 > gpurun_out/march_sweep_$dt.json 2> gpurun_out/march_sweep_$dt.log
  r=$?; echo "sweep $dt rc=$r"; cat gpurun_out/march_sweep_$dt.json; if [ $r -ne 0 ]; then exit $r; fi
done
rm -rf gpurun_out/march_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/march_trace/bf16 -o m --output-format csv -- python3 tools/march_bench.py --dtype bf16 --schedule 12x2_klow8_t0.9 > gpurun_out/march_trace_bf16.log 2>&1
r=$?; echo "trace rc=$r"
exit $rc
