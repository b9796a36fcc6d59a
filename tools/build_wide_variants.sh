#!/bin/bash
# variants of the bf16x3 forward objects (mlp_p2_0 training, p2_1 inference, p2_4 bf16x3f training) into vgpu/<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  B=/tmp/nerf_var_$name
  rm -rf $B; cp -rp $ROOT/build/nerf_amd $B; touch $B/*.o
  rm -f $B/mlp_p2_0.o $B/mlp_p2_1.o $B/mlp_p2_4.o
  make -C $ROOT/nerf-replication_amd/csrc -j3 BUILD=$B OUT=$ROOT/vgpu/$name.so EXTRA="$defs" > /tmp/nerf_var_$name.log 2>&1 &
done
wait
ls -la $ROOT/vgpu
