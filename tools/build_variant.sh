#!/bin/bash
# Tuning aid: build a variant of liblssp_amd.so whose linesweep.hip (or the
# sources named in $VSRC, e.g. VSRC="kernels capi") is compiled with extra defines, into
# build/<name>.so (load it with LSSP_AMD_LIB=...).
#   tools/build_variant.sh <name> -DLINE_DH_OVERRIDE=6 ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
make -s -C "$ROOT/lssp_amd/csrc"
OBJ=$ROOT/lssp_amd/lib/obj
mkdir -p "$ROOT/build/$name"
FLAGS="-O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I$ROOT/include -I/opt/rocm/include"
objs=$(ls $OBJ/*.o)
vobjs=""
for SRC in ${VSRC:-linesweep}; do  # VSRC: one or more of kernels linesweep capi ... (.hip or .cpp)
  f=$(ls "$ROOT/lssp_amd/csrc/$SRC".hip "$ROOT/lssp_amd/csrc/$SRC".cpp 2>/dev/null | head -1)
  /opt/rocm/bin/hipcc $FLAGS "$@" -c "$f" -o "$ROOT/build/$name/$SRC.o" 2>/dev/null
  objs=$(echo "$objs" | grep -v "/$(basename "$f").o")
  vobjs="$vobjs $ROOT/build/$name/$SRC.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/build/$name.so" $objs $vobjs \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$ROOT/build/$name.so"
