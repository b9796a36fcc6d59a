#!/bin/bash
# Round 6: the wide bf16 dX (PBF16W) against the 32x32 one (vgpu/cur.so = the build before it)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
for dt in bf16 bf16x3f; do
  timeout -k 10 300 python tools/dx_compare.py --dtype $dt --libs vgpu/cur.so,vgpu/wdx16.so > $O/wdx16_cmp_$dt.json 2> $O/wdx16_cmp_$dt.err || exit $?
  cat $O/wdx16_cmp_$dt.json
done
for dt in bf16 bf16x3f; do
  timeout -k 10 300 python tools/mlp_bench.py --dtype $dt --libs vgpu/cur.so,vgpu/wdx16.so --M 524288 --reps 5 --rounds 7 >> $O/wdx16_ab.json 2>> $O/wdx16_ab.err || exit $?
done
cat $O/wdx16_ab.json
