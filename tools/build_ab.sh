#!/bin/bash
# Build libencx.so of a git revision for an on-box A/B: tools/build_ab.sh <rev> <name>
#   -> encodec-pytorch_amd/ab/<name>.so (git-ignored; travels with gpurun). Pick it in a bench
#   variant with ENCX_LIB=encodec-pytorch_amd/ab/<name>.so (encx._lib then only warns that its
#   build id differs from the sources in the tree).
set -eu
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
git -C "$root" archive "$rev" encodec-pytorch_amd include | tar -x -C "$tmp"
make -C "$tmp/encodec-pytorch_amd" -j8 > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
mkdir -p "$root/encodec-pytorch_amd/ab"
cp "$tmp/encodec-pytorch_amd/encx/libencx.so" "$root/encodec-pytorch_amd/ab/$name.so"
echo "built $rev -> encodec-pytorch_amd/ab/$name.so"
