set -o pipefail
mkdir -p gpurun_out/tail3
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tail3/pytest.log 2>&1 || { tail -30 gpurun_out/tail3/pytest.log; exit 1; }
tail -2 gpurun_out/tail3/pytest.log
timeout -k 10 300 python tools/tail_bench.py 216 100 1 > gpurun_out/tail3/ab.txt 2>&1
