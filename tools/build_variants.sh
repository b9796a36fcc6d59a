#!/bin/bash
# Build experimental variants of libnerf_amd.so (mlp.hip with -D overrides) into variants/<name>.so
# usage: tools/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "..." ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/nerf-replication_amd/csrc
make -C $CS -j8 > /dev/null
mkdir -p $ROOT/variants
pids=()
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  (
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include $defs -c ${SRC:-$CS/mlp.hip} -o /tmp/var_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/variants/$name.so /tmp/var_$name.o \
      $ROOT/build/nerf_amd/sampling.hip.o $ROOT/build/nerf_amd/grid.hip.o $ROOT/build/nerf_amd/optim.hip.o $ROOT/build/nerf_amd/metrics.hip.o $ROOT/build/nerf_amd/errors.cpp.o
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la $ROOT/variants
