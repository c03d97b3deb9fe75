#!/bin/bash
# diagnostics: build libc3hlac_mi355x.so with extra -D flags into lib/variants/<name>.so
# usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2"   (select with C3HLAC_LIB=...)
set -e
cd "$(dirname "$0")/../mapping-private_amd"
NAME=$1; shift
B=build/variants/$NAME; mkdir -p $B lib/variants
pids=()
for f in capi voxelize c3hlac search pipeline colour pcdio pca ingest rsd dist; do
  rm -f $B/$f.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $* -c csrc/$f.hip -o $B/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $NAME: compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/variants/$NAME.so $B/*.o -ldl
