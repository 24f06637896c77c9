#!/bin/bash
# Tuning aid (GPU box): line-sweep timings of the default library and of
# variant builds (tools/build_variant.sh) -- tools/gpu_exp.sh [N] variant ...
N=${1:-216}; shift
for v in default "$@"; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/line_diag.py "$N" 0,0 || echo "variant $v failed"
done
