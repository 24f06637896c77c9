#!/bin/bash
# Tuning aid (GPU box): BiCGSTAB+ILU(0) 216^3 it/s over LSSP_AMD_SPMV_NTV x
# LSSP_AMD_GATHER_EW, alternated in one session, plus kernel stats of ntv=0.
set -o pipefail
O=gpurun_out/${1:-ntvgew}; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for v in "1 1" "0 1" "1 0" "0 0"; do
    set -- $v
    echo "== ntv=$1 gew=$2" >> $O/ab.txt
    LSSP_AMD_SPMV_NTV=$1 LSSP_AMD_GATHER_EW=$2 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
LSSP_AMD_SPMV_NTV=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o b -- python3 $R/bench.py --steps 30 --no-cpu --config4-steps 0 > $R/$O/prof.log 2>&1 || exit 1
