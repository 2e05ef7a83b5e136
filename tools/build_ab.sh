#!/bin/bash
# A/B variant of libsdnroute.so: the current sources with extra -D flags.
# Usage: bash tools/build_ab.sh NAME -DFLAG...   -> tools/ab/libsdnroute_NAME.so
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/sdn-mpi-router_amd/csrc
OUT=$ROOT/tools/ab/$NAME; mkdir -p $OUT
pids=()
for f in capi dfs shortest apsp routes ecmp incremental; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function "$@" -c -o $OUT/$f.o $C/$f.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o $ROOT/tools/ab/libsdnroute_$NAME.so $OUT/*.o -Wl,-rpath,/opt/rocm/lib
rm -rf $OUT
echo built tools/ab/libsdnroute_$NAME.so
