#!/bin/bash
# Build the library with ONE source file compiled under extra flags, for an on-box A/B of a
# compile-time constant: tools/build_flag_variant.sh <source stem> <name> <flags...>
#   e.g. tools/build_flag_variant.sh conv1d sper8 -DENCX_SPER=8 -> encodec-pytorch_amd/ab/sper8.so
# (run `make -C encodec-pytorch_amd` first: the other objects are taken from build/).
set -eu
stem=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
cd "$root/encodec-pytorch_amd"
mkdir -p ab build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Wno-unused-function \
    -Wno-unused-variable "$@" -c "csrc/$stem.hip" -o "build/var/$stem.$name.o"
objs="build/buildid.o"
for f in csrc/*.hip; do
    b=$(basename "$f" .hip)
    [ "$b" != "$stem" ] && objs="$objs build/$b.o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "ab/$name.so" $objs "build/var/$stem.$name.o"
echo "built ab/$name.so ($stem.hip with $*)"
