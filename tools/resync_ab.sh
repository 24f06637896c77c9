#!/bin/bash
# Tuning aid (GPU box): the sweeps' resync episode without (default) and with
# the wait for the furthest step in flight (build/far.so: k_line2, build/ffar.so:
# k_linef) -- apply timings (bitwise-checked), 216^3 bench A/B.  OUT
set -o pipefail
O=gpurun_out/${1:-resync}; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default far; do
    echo "== ilu0 $v" >> $O/ab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep -v amdgpu >> $O/ab.txt || exit 1
    LSSP_AMD_LIB=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
  for v in default ffar; do
    echo "== ilu1 $v" >> $O/ab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LINE_DIAG_LEVEL=1 LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep -v amdgpu >> $O/ab.txt || exit 1
  done
done
