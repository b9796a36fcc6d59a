# round 3: torch-order CDF normaliser (sample_pdf tests, render_video golden frames, trained-net
# parity), then the 2-rank prefetch/all-reduce overlap trace
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trained.py -m gpu -v -s -k "pdf or searchsorted or trained or video or render or grad" \
  --maxfail=6 --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r3d_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/dp_overlap_trace.py > gpurun_out/dp_overlap.log 2>&1
r=$?; tail -40 gpurun_out/dp_overlap.log; echo "overlap rc=$r"
rm -f gpurun_out/dp_overlap_trace_rank*.json.gz
exit $rc
