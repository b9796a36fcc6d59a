#!/bin/bash
# Round 6: knob sweep of the wide bf16x3 forward (vgpu/w_*.so) + the bench line of the default build
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
O=gpurun_out/r6
libs=vgpu/wide.so$(for f in vgpu/w_*.so; do printf ",%s" $f; done)
for dt in bf16x3f bf16x3; do
  timeout -k 10 400 python tools/mlp_bench.py --dtype $dt --libs $libs --M 524288 --reps 5 --rounds 5 >> $O/tune.json 2>> $O/tune.err || exit $?
done
echo tune done
timeout -k 10 600 python bench.py > $O/bench_wide.json 2> $O/bench_wide.err
rc=$?
tail -c 600 $O/bench_wide.json
exit $rc
