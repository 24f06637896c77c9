#!/bin/bash
# Tuning aid (GPU box): packet-sweep traces (tools/pk6_trace.py) of the default
# library and of variant builds (tools/build_variant.sh, VSRC=trisolve) --
#   tools/pk6_exp.sh [N] variant ...
N=${1:-128}; shift
for v in default "$@"; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 200 python tools/pk6_trace.py "$N" 60 ilut 2>&1 | grep -v amdgpu.ids || echo "variant $v failed"
done
