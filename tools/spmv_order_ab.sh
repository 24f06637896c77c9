#!/bin/bash
# Tuning aid (GPU box): the product's block order and non-temporal vector
# operands (LSSP_AMD_SPMV_ORDER = column-group width in blocks, 0 = natural;
# LSSP_AMD_SPMV_NTV, kernels.hip) on the 512^3 solve and its 8-rank slab
# projection -- tools/spmv_order_ab.sh OUT [W]
OUT=${1:-gpurun_out/spmv_order}; W=${2:-128}; mkdir -p "$OUT"
for v in "0 0" "$W 0" "0 1" "$W 1"; do
  set -- $v
  echo "== order=$1 ntv=$2" | tee -a "$OUT/ab.txt"
  LSSP_AMD_SPMV_ORDER=$1 LSSP_AMD_SPMV_NTV=$2 timeout -k 10 280 python tools/project_ranks.py --grid 512 --ranks 1,8 --steps 20 >> "$OUT/ab.txt" || exit 1
done
