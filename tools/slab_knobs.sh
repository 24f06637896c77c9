#!/bin/bash
# Tuning aid (GPU box): the 8-rank 512^3 slab's BiCGSTAB iteration (tools/
# project_ranks.py --ranks 8) for the default library and variant builds -- OUT name ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    echo "== $v" >> $O/slab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LSSP_AMD_LIB=$L timeout -k 10 200 python tools/project_ranks.py --grid 512 --ranks 8 --steps 20 >> $O/slab.txt || exit 1
  done
done
