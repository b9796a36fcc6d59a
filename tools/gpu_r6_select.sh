#!/bin/bash
# Round 6: the selective coarse pass of the split-bf16 renders: CDF calibration, kernel test, full-frame test
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
timeout -k 10 300 python tools/cdf_sensitivity.py --dtype bf16x3 --out $O/cdf_sensitivity.json > $O/cdf_sensitivity.log 2>&1 || { tail -5 $O/cdf_sensitivity.log; exit 1; }
tail -c 1200 $O/cdf_sensitivity.json; echo
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fragile or composite_pdf" -x -q --timeout 300 --timeout-method thread > $O/select_tests.log 2>&1 || { tail -20 $O/select_tests.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullframe.py -k "config2" -x -q -s --timeout 300 --timeout-method thread >> $O/select_tests.log 2>&1
rc=$?
grep -E "fragile|render bf16x3|passed|failed|Error" $O/select_tests.log | tail -12
exit $rc
