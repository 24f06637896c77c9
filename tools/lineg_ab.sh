#!/bin/bash
# k_lineg timing variants (results of nowait/nodma are wrong: timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g3
for v in base; do
  L=; [ $v != base ] && L=$PWD/build/$v.so
  LSSP_AMD_LIB=$L timeout -k 10 120 python -u tools/lineg_bench.py --lines > gpurun_out/g3/$v.log 2>&1 || exit 1
  echo "$v $(grep one-workgroup gpurun_out/g3/$v.log | head -2 | cut -c1-150 | tr '\n' ' ')"
done
