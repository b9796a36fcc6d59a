#!/bin/bash
# Round 6: the wide dX (DxWave16, PF32W / PBF3W) against the 32x32 one (vgpu/cur.so = the build before it)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
for dt in fp32 bf16x3; do
  timeout -k 10 300 python tools/dx_compare.py --dtype $dt --libs vgpu/cur.so,vgpu/wdx.so > $O/wdx_cmp_$dt.json 2> $O/wdx_cmp_$dt.err || exit $?
  cat $O/wdx_cmp_$dt.json
done
for dt in fp32 bf16x3; do
  timeout -k 10 300 python tools/mlp_bench.py --dtype $dt --libs vgpu/cur.so,vgpu/wdx.so --M 524288 --reps 3 --rounds 5 >> $O/wdx_ab.json 2>> $O/wdx_ab.err || exit $?
done
cat $O/wdx_ab.json
