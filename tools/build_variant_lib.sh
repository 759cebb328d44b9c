#!/bin/bash
# Build libprodiff_hip.so of the WORKING TREE with extra compile flags for fastdiff.hip, wavenet.hip and nsf_hifigan.hip into
# tools/bin/lib_<name>.so (same-box A/B: PRODIFF_HIP_LIB=tools/bin/lib_<name>.so).  The other
# objects are reused from the in-tree build.   usage: tools/build_variant_lib.sh <name> "<flags>"
set -e
NAME=$1; EXTRA=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d)
mkdir -p "$D/prodiff_amd"
cp -rp "$R/include" "$D/"
cp -rp "$R/prodiff_amd/csrc" "$D/prodiff_amd/"
rm -f "$D/prodiff_amd/csrc/build/fastdiff.o" "$D/prodiff_amd/csrc/build/wavenet.o" "$D/prodiff_amd/csrc/build/nsf_hifigan.o"
make -C "$D/prodiff_amd/csrc" -j8 CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $EXTRA" > "$D/build.log" 2>&1 || { tail -20 "$D/build.log"; exit 1; }
mkdir -p "$R/tools/bin"
cp "$D/prodiff_amd/libprodiff_hip.so" "$R/tools/bin/lib_$NAME.so"
rm -rf "$D"
echo "tools/bin/lib_$NAME.so"
