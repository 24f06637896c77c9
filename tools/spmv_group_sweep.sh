#!/bin/bash
# Tuning aid (GPU box): y = A x with the column-group block order
# (LSSP_AMD_SPMV_ORDER = group width in blocks, 0 = natural) -- OUT
OUT=${1:-gpurun_out/spmv_group}; mkdir -p "$OUT"
run() { echo "== W=$W $*" >> "$OUT/sweep.txt"; LSSP_AMD_SPMV_ORDER=$W timeout -k 10 200 python tools/bench_spmv.py "$@" >> "$OUT/sweep.txt" || exit 1; }
for W in 0 1 4 16 32 64 128 256 0; do run --grid 512 --nz 64; done
for W in 0 32 128; do run --grid 512; done
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for W in 32 128; do
  LSSP_AMD_SPMV_ORDER=$W timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$OUT/mv_W$W" -o p -- python3 "$R/tools/bench_spmv.py" --grid 512 --nz 64 --reps 10 > "$R/$OUT/mv_W$W.log" 2>&1 || exit 1
done
