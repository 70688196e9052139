#!/bin/bash
# Build an A/B variant of libkair_hip.so: tools/build_variant.sh <out.so> <source.hip> <extra hipcc flags...>
# (the named source recompiled with the flags, every other object from kair_amd/build/)
set -e
OUT=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/kair_amd/csrc -I $R/include -Wno-unused-result -Wno-inline-asm \
  -munsafe-fp-atomics "$@" -c $R/kair_amd/csrc/$SRC -o $T/v.o
OBJS=$(ls $R/kair_amd/build/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $T/v.o -o $OUT
rm -rf $T
echo built $OUT
