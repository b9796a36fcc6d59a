#!/bin/bash
# Build experimental variants of libnerf_amd.so (compile-time -D overrides) into variants/<name>.so
# usage: tools/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "..." ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/nerf-replication_amd/csrc
mkdir -p $ROOT/variants
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  make -C $CS -j8 BUILD=/tmp/nerf_var_$name OUT=$ROOT/variants/$name.so EXTRA="$defs" > /tmp/nerf_var_$name.log 2>&1
done
ls -la $ROOT/variants
