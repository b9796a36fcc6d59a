#!/bin/bash
# Build experimental variants of libnerf_amd.so (compile-time -D overrides) into variants/<name>.so
#   tools/build_variants.sh [-o "mlp_p2_0 mlp_p2_2"] name1 "-DFOO=1 -DBAR=2" name2 "..." ...
# -o: rebuild only these objects (the rest are copied from the default build in build/nerf_amd,
# which must be up to date); default: every object.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/nerf-replication_amd/csrc
ONLY=""
if [ "$1" = "-o" ]; then ONLY=$2; shift 2; fi
mkdir -p $ROOT/variants
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  B=/tmp/nerf_var_$name
  rm -rf $B
  if [ -n "$ONLY" ]; then
    cp -rp $ROOT/build/nerf_amd $B
    touch $B/*.o  # (newer than any edited source: only the listed objects are rebuilt)
    for o in $ONLY; do rm -f $B/$o.o; done
  fi
  make -C $CS -j8 BUILD=$B OUT=$ROOT/variants/$name.so EXTRA="$defs" > /tmp/nerf_var_$name.log 2>&1 || { tail -20 /tmp/nerf_var_$name.log; exit 1; }
done
ls -la $ROOT/variants
