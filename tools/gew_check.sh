#!/bin/bash
# Tuning aid (GPU box): the fused p / s gathers (LSSP_AMD_GATHER_EW) and the
# LDS-transposed k_line2 gather (variants build/run8.so, run16.so: LRHS2_RUN)
# -- parity subset, bench A/B, kernel stats.  tools/gew_check.sh OUT
set -o pipefail
O=gpurun_out/${1:-gew}; mkdir -p $O; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tail.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for g in 1 0; do
    echo "== gew=$g" >> $O/ab.txt
    LSSP_AMD_GATHER_EW=$g timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
  for v in run16 run8; do
    echo "== $v gew=0" >> $O/ab.txt
    LSSP_AMD_LIB=$R/build/$v.so LSSP_AMD_GATHER_EW=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for g in 0 1; do
  LSSP_AMD_GATHER_EW=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof$g -o b -- python3 $R/bench.py --steps 30 --no-cpu --config4-steps 0 > $R/$O/prof$g.log 2>&1 || exit 1
done
