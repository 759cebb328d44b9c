#!/bin/bash
# Build libprodiff_hip.so of a git revision into tools/bin/lib_<rev>.so (for same-box A/B runs:
# PRODIFF_HIP_LIB=tools/bin/lib_<rev>.so python bench.py ...).   usage: tools/build_rev_lib.sh <rev>
set -e
REV=$1
R=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d)
git -C "$R" archive "$REV" prodiff_amd/csrc include | tar -x -C "$D"
make -C "$D/prodiff_amd/csrc" -j8 > /dev/null
mkdir -p "$R/tools/bin"
cp "$D/prodiff_amd/libprodiff_hip.so" "$R/tools/bin/lib_$REV.so"
rm -rf "$D"
echo "tools/bin/lib_$REV.so"
