#!/bin/bash
# Build a compile-time variant of the library for an A/B (tools/gpu_ab_lib.sh):
#   tools/build_variant.sh TAG "-DNAME=VALUE ..." ["capi.o other.o"]
#   -> jwave_amd/lib/ab_TAG.so
# Objects start as a copy of the default build; the listed objects (default:
# all) are rebuilt with the defines.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; DEFS=$2; OBJ=${3:-}
make -s -C $R/jwave_amd/csrc -j8 >/dev/null
rm -rf $R/build/obj_$TAG; cp -a $R/build/obj $R/build/obj_$TAG
if [ -n "$OBJ" ]; then for o in $OBJ; do rm -f $R/build/obj_$TAG/$o; done; else rm -f $R/build/obj_$TAG/*.o; fi
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function -MMD -MP $DEFS"
make -s -C $R/jwave_amd/csrc -j8 OBJDIR=../../build/obj_$TAG LIB=../lib/ab_$TAG.so CXXFLAGS="$FLAGS" 2>&1 | grep -E "error" || true
ls -la $R/jwave_amd/lib/ab_$TAG.so
