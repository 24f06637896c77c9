#!/bin/bash
# GPU check of the packet sweeps (ILUT / general factors) and a config-3 timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "ilut or ILUT or packet or pk6 or general or golden" -x -q --timeout 200 --timeout-method thread > gpurun_out/p6/pytest.log 2>&1 || { tail -30 gpurun_out/p6/pytest.log; exit 1; }
tail -2 gpurun_out/p6/pytest.log
if [ "$1" = trace ]; then
  timeout -k 10 300 python -u tools/pk6_trace.py 128 60 ilut > gpurun_out/p6/trace.txt 2>&1 || { tail -20 gpurun_out/p6/trace.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/p6/trace.txt | tail -12
fi
