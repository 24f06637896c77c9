#!/bin/bash
# GPU check of the one-workgroup 2-D sweeps (k_lineg) and the tests around them
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g2
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tail.py tests/test_gpu_fullsize.py -k "ilu1 or tail or 2d" -x -q --timeout 120 --timeout-method thread > gpurun_out/g2/pytest.log 2>&1 || { tail -40 gpurun_out/g2/pytest.log; exit 1; }
tail -2 gpurun_out/g2/pytest.log
