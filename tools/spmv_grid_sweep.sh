#!/bin/bash
# Tuning aid (GPU box): y = A x on 7-pt grids of several sizes under the SpMV
# block-order knobs -- tools/spmv_grid_sweep.sh OUT "GRIDS" "ORDERS" "STREAMS" ["SKEWS"]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for g in $2; do for o in $3; do for k in $4; do for w in ${5:-0}; do
  echo "== grid $g order $o streams $k skew $w" >> $O/spmv.txt
  LSSP_AMD_SPMV_ORDER=$o LSSP_AMD_SPMV_STREAMS=$k LSSP_AMD_SPMV_SKEW=$w timeout -k 10 120 python tools/bench_spmv.py --grid $g --reps 100 >> $O/spmv.txt 2>/dev/null || exit 1
done; done; done; done
