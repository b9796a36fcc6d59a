# round 3: new DP / prefetch tests, bf16 rounding-model pin, march skip at res 128-1024, trained-net grads,
# device-count march; then (only if the tests ended normally: pass or assertion failures) a march
# schedule sweep, a march kernel trace and a short bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_eval.py tests/test_gpu_kernels.py tests/test_gpu_trained.py tests/test_gpu_render.py -m gpu -v -s \
  --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3a_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for dt in bf16 fp32; do
  timeout -k 10 300 python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9,12x2_klow4_t0.9,12x2_klow2_t0.9,12x2_klow8_t0.9_sync8,12x2_klow4_t0.9_sync8,12x2_klow2_t0.9_sync8 > gpurun_out/march_sweep_$dt.json 2> gpurun_out/march_sweep_$dt.log
  r=$?; echo "sweep $dt rc=$r"; cat gpurun_out/march_sweep_$dt.json; if [ $r -ne 0 ]; then exit $r; fi
done
rm -rf gpurun_out/march_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/march_trace/bf16 -o m --output-format csv -- python3 tools/march_bench.py --dtype bf16 --schedule 12x2_klow8_t0.9 > gpurun_out/march_trace_bf16.log 2>&1
r=$?; if [ $r -ne 0 ]; then echo "march trace rc=$r"; exit $r; fi
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.log
r=$?; echo "bench rc=$r"; tail -c 400 gpurun_out/r3a_bench.json
exit $rc
