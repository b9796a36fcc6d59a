#!/bin/bash
# Parallel variant builds: copies of the default build (build/nerf_amd, up to date) with the listed objects
# rebuilt under extra -D flags, each linked to ab/<name>.so.
#   tools/build_variants_par.sh "mlp_p2_4 mlp_p2_1" name1 "-DFOO=1" name2 "-DBAR=2" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/nerf-replication_amd/csrc
ONLY=$1; shift
mkdir -p $ROOT/ab
pids=()
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  B=/tmp/nerf_var_$name
  rm -rf $B; cp -rp $ROOT/build/nerf_amd $B; touch $B/*.o
  for o in $ONLY; do rm -f $B/$o.o; done
  (make -C $CS -j${VJ:-4} BUILD=$B OUT=$ROOT/ab/$name.so EXTRA="$defs" > /tmp/nerf_var_$name.log 2>&1 || echo "FAILED $name") &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la $ROOT/ab
