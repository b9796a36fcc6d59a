# round 3: the entry-point workflow test, then the fp32 200k-step config-3 curve (part)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_entrypoints.py -m gpu -v -s --timeout 380 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/r3h_tests.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_psnr200k.sh fp32
r=$?; if [ $r -ne 0 ]; then exit $r; fi
exit $rc
