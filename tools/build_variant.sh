#!/bin/bash
# Variant build of libsvla.so: tools/build_variant.sh NAME "EXTRA flags" src1.hip [src2.hip ...]
# Reuses the product objects for every other source; the variant library lands in diag/libsvla_NAME.so.
set -e
NAME=$1; FLAGS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/obj_$NAME
mkdir -p $OBJ $R/diag
cp -p $R/build/obj/*.o $OBJ/
for s in "$@"; do rm -f $OBJ/${s%.hip}.o; done
make -s -C $R/spatialvla_amd/csrc -j8 OUT=$R/diag/libsvla_$NAME.so OBJDIR=$OBJ EXTRA="$FLAGS"
echo built diag/libsvla_$NAME.so
