#!/bin/bash
# Tuning aid (GPU box): standalone y = A x rate across grid shapes (cubes and
# z-slabs of the block-Jacobi blocks) -- tools/spmv_shape_sweep.sh OUT
OUT=${1:-gpurun_out/spmv_shape}; mkdir -p "$OUT"
run() { echo "== $*" >> "$OUT/sweep.txt"; timeout -k 10 200 python tools/bench_spmv.py "$@" >> "$OUT/sweep.txt" || exit 1; }
run --grid 216
run --grid 512 --nz 64
run --grid 500 --nz 67
run --grid 520 --nz 62
run --grid 432 --nz 90
run --grid 512 --nz 128
run --grid 256 --nz 256
run --grid 512 --nz 64
LSSP_AMD_SPMV_ORDER=1 run --grid 512 --nz 64
LSSP_AMD_SPMV_STREAMS=64 run --grid 512 --nz 64
run --grid 512
