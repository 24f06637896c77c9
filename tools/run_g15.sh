# GPU box: block-Jacobi ILU(1) on P ranks through the line sweeps; ILU(1) parity and timing
# after the run-based rhs gather (gpurun_out/g15/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "ilu1" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dist.py -k "ilu1" > $O/dist.log 2>&1 || { tail -30 $O/dist.log; exit 1; }
tail -4 $O/dist.log
for i in 1 2; do LINE_DIAG_LEVEL=1 timeout -k 10 200 python tools/line_diag.py 128 0 2>&1 | grep '^{' || exit 1; done | tee $O/ilu1_128.txt
