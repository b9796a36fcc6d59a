# round 3: one-pass march gather (tests: brute-force gather, trained-net march exact query count), sweep
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trained.py tests/test_gpu_render.py -m gpu -v -k "march or accelerated or grid" \
  --maxfail=4 --timeout 300 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3f_tests.log | tail -3; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r3f_tests.log | head; exit $rc; fi
for dt in bf16 fp32; do
  timeout -k 10 300 python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9,12x2_klow8_t0.9_2pass,12x2_klow8_t0.9_g4,12x2_klow8_t0.9_g6,12x2_klow8_t0.9_g8,12x2_klow8_t0.9_g10,12x2_klow4_t0.9_g6,16x2_klow8_t0.9_g6 > gpurun_out/march_sweep3_$dt.json 2> gpurun_out/march_sweep3_$dt.log
  r=$?; echo "sweep $dt rc=$r"; cat gpurun_out/march_sweep3_$dt.json; if [ $r -ne 0 ]; then exit $r; fi
done
exit $rc
