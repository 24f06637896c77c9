#!/bin/bash
# Tuning aid: build a variant of liblssp_amd.so whose linesweep.hip (or
# $VSRC, e.g. VSRC=kernels) is compiled with extra defines, into
# build/<name>.so (load it with LSSP_AMD_LIB=...).
#   tools/build_variant.sh <name> -DLINE_DH_OVERRIDE=6 ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
make -s -C "$ROOT/lssp_amd/csrc"
OBJ=$ROOT/lssp_amd/lib/obj
mkdir -p "$ROOT/build/$name"
FLAGS="-O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I$ROOT/include -I/opt/rocm/include"
SRC=${VSRC:-linesweep}
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$ROOT/lssp_amd/csrc/$SRC.hip" -o "$ROOT/build/$name/$SRC.o" 2>/dev/null
objs=$(ls $OBJ/*.o | grep -v "/$SRC.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/build/$name.so" $objs "$ROOT/build/$name/$SRC.o" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$ROOT/build/$name.so"
