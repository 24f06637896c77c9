# GPU box: ILU(1) line sweeps -- parity first (gpurun_out/g8/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ilu1 or trisolve_sweeps" > $O/parity.log 2>&1
rc=$?; tail -25 $O/parity.log; exit $rc
