#!/bin/bash
# Tuning aid (GPU box): 216^3 BiCGSTAB+ILU(1) it/s (tools/tail_bench.py, tail on)
# of the default library and variant builds, alternated -- OUT name ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    echo "== $v" >> $O/ab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LSSP_AMD_LIB=$L TAIL_MODES=1 timeout -k 10 300 python tools/tail_bench.py 216 100 1 2>&1 | grep -v amdgpu >> $O/ab.txt || exit 1
  done
done
