#!/bin/bash
# Tuning aid (GPU box): HBM bytes per launch (FETCH_SIZE / WRITE_SIZE passes)
# of the 8-rank 512^3 slab solve and of the standalone slab product --
# tools/slab_pmc.sh OUT
OUT=${1:-gpurun_out/slab_pmc}; mkdir -p "$OUT"; R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$R/$OUT/solve_$c" -o p -- python3 "$R/tools/project_ranks.py" --grid 512 --ranks 8 --steps 5 > "$R/$OUT/solve_$c.log" 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$R/$OUT/mv_$c" -o p -- python3 "$R/tools/bench_spmv.py" --grid 512 --nz 64 --reps 10 > "$R/$OUT/mv_$c.log" 2>&1 || exit 1
done
