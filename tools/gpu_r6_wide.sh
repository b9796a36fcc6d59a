#!/bin/bash
# Round 6: the wide (16x16x32, two waves per SIMD) bf16x3 forward against the 32x32 one (vgpu/def.so)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
for dt in bf16x3f bf16x3; do
  timeout -k 10 300 python tools/race_diag.py --dtype $dt --libs vgpu/def.so,vgpu/wide.so --runs 2 > $O/wide_$dt.json 2> $O/wide_$dt.err || exit $?
done
echo diag done
for dt in bf16x3f bf16x3; do
  timeout -k 10 300 python tools/mlp_bench.py --dtype $dt --libs vgpu/def.so,vgpu/wide.so --M 524288 --reps 5 --rounds 7 >> $O/wide_ab.json 2>> $O/wide_ab.err || exit $?
done
echo ab done
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trained.py tests/test_gpu_fullframe.py -k "bf16x3" -x -q --timeout 300 --timeout-method thread > $O/wide_tests.log 2>&1
rc=$?
tail -5 $O/wide_tests.log
exit $rc
