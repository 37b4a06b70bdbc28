#!/bin/bash
# Diagnostic A/B builds: recompile ONE source of libsvla with extra -D flags and link it with the main build's other
# objects: tools/build_variant.sh <source.hip> <out.so> -DKNOB=VALUE ...
set -e
src=$1; out=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/spatialvla_amd/csrc
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc "$@" -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable \
  -munsafe-fp-atomics -ffp-contract=fast -c "$C/$src" -o "$tmp/${src%.hip}.o"
objs=$(ls "$R"/build/obj/*.o | grep -v "/${src%.hip}.o$")
/opt/rocm/bin/hipcc -shared -fPIC -Wl,-Bsymbolic --offload-arch=gfx950 $objs "$tmp/${src%.hip}.o" -o "$out"
rm -rf "$tmp"
