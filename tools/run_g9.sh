# GPU box: ILU(1) line sweeps -- full-size parity and the general-ilu bench (gpurun_out/g9/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g9; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k ilu1 > $O/fullsize.log 2>&1 && \
timeout -k 10 600 python -u tools/bench_configs.py general-ilu --ref-iters 0 > $O/general_ilu.jsonl 2> $O/general_ilu.err
rc=$?; tail -5 $O/fullsize.log; cat $O/general_ilu.jsonl | cut -c1-700; exit $rc
