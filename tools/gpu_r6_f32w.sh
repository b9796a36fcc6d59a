#!/bin/bash
# Round 6: the wide fp32 training forward (PF32W) against PF32's (vgpu/cur.so = the build before it)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
timeout -k 10 300 python tools/race_diag.py --dtype fp32 --libs vgpu/cur.so,vgpu/f32w.so --runs 2 --M 524288 > $O/f32w_diag.json 2> $O/f32w_diag.err || exit $?
echo diag done
timeout -k 10 300 python tools/mlp_bench.py --dtype fp32 --libs vgpu/cur.so,vgpu/f32w.so --M 524288 --reps 3 --rounds 5 > $O/f32w_ab.json 2> $O/f32w_ab.err || exit $?
echo ab done
cat $O/f32w_ab.json
