#!/bin/bash
# Tuning aid (GPU box): 216^3 bench it/s with environment settings A/B'd,
# alternated -- tools/env_ab.sh OUT "VAR=val ..." "VAR=val ..." ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2 3; do
  for v in "" "$@"; do
    echo "== ${v:-default}" >> $O/ab.txt
    env $v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
done
