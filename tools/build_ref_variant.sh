#!/bin/bash
# diagnostics: build libc3hlac_mi355x.so from a git revision's csrc/ (A/B against the
# working tree) into lib/variants/<name>.so.  usage: tools/build_ref_variant.sh NAME REV "-DFLAGS"
set -e
cd "$(dirname "$0")/../mapping-private_amd"
NAME=$1; REV=$2; shift 2
S=build/variants/src_$NAME; B=build/variants/$NAME
rm -rf $S; mkdir -p $S $B lib/variants
(cd .. && git archive $REV mapping-private_amd/csrc include) | tar -x -C $S
pids=()
for f in capi voxelize c3hlac search pipeline colour pcdio pca ingest rsd dist; do
  rm -f $B/$f.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    $* -c $S/mapping-private_amd/csrc/$f.hip -o $B/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $NAME: compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/variants/$NAME.so $B/*.o -ldl
