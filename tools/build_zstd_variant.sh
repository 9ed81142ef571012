#!/bin/bash
# Builds a zstd A/B variant of the product library: okv_zstd.hip (or the
# file given by ZST_SRC) with extra defines, linked with the other product
# objects from objectkv_amd/build, into tools/ab/r5/lib_zst<NAME>.so.
# usage: [ZST_SRC=path] tools/build_zstd_variant.sh NAME [-DFOO=1 ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
B=$R/objectkv_amd/build; D=$R/tools/ab/r5; mkdir -p "$D"
SRC=${ZST_SRC:-$R/objectkv_amd/csrc/okv_zstd.hip}
# (no make here: the working tree may hold the variant's source, and make would
# rebuild the product library from it; the other objects come from the last
# product build)
for o in okv_decode okv_encode okv_zstd okv_merge okv_host okv_reader; do
  [ -f "$B/$o.o" ] || { echo "missing $B/$o.o: run make -C objectkv_amd/csrc first" >&2; exit 1; }
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I"$R/include" \
  -I"$R/objectkv_amd/csrc" "$@" -c "$SRC" -o "$D/zst_$N.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$D/lib_zst$N.so" \
  "$D/zst_$N.o" "$B/okv_decode.o" "$B/okv_encode.o" "$B/okv_merge.o" "$B/okv_host.o" "$B/okv_reader.o"
echo "built $D/lib_zst$N.so"
