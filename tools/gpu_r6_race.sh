#!/bin/bash
# Round 6: the finish-part race, settled (tools/race_diag.py), the cost of the fix (tools/mlp_bench.py --libs)
# and the determinism / mask tests, on one GPU box.  Variant builds in vgpu/ (built here beforehand).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
timeout -k 10 300 python tools/race_diag.py --libs vgpu/def.so,vgpu/p2n.so,vgpu/r5p2.so,vgpu/r5p8.so,vgpu/r5def.so --runs 3 > $O/race_bf16.json 2> $O/race_bf16.err || exit $?
echo race_bf16 done
timeout -k 10 300 python tools/race_diag.py --dtype bf16x3 --libs vgpu/def.so,vgpu/bf3p4.so,vgpu/r5def.so --runs 3 > $O/race_bf16x3.json 2> $O/race_bf16x3.err || exit $?
timeout -k 10 300 python tools/race_diag.py --dtype bf16x3f --libs vgpu/def.so,vgpu/bf3p4.so,vgpu/r5def.so --runs 3 > $O/race_bf16x3f.json 2> $O/race_bf16x3f.err || exit $?
echo race_x3 done
for dt in bf16 bf16x3f fp32; do
  timeout -k 10 300 python tools/mlp_bench.py --dtype $dt --libs vgpu/r5def.so,vgpu/def.so,vgpu/p2n.so --M 524288 --reps 5 --rounds 7 >> $O/ab_fix.json 2>> $O/ab_fix.err || exit $?
done
timeout -k 10 300 python tools/mlp_bench.py --dtype bf16x3 --libs vgpu/r5def.so,vgpu/def.so,vgpu/bf3p4.so --M 524288 --reps 5 --rounds 7 >> $O/ab_fix.json 2>> $O/ab_fix.err || exit $?
echo ab done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "deterministic or ragged" -x -q --timeout 200 --timeout-method thread > $O/det_tests.log 2>&1 || exit $?
echo det done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullframe.py -x -q -s --timeout 300 --timeout-method thread > $O/fullframe.log 2>&1
rc=$?
tail -3 $O/fullframe.log
exit $rc
