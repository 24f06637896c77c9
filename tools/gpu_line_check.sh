# line-sweep check on the GPU box: a small bitwise apply, the ILU/solver parity
# subset, then timings at 216^3 (tuning aid)
set -o pipefail
timeout -k 10 60 python tools/line_diag.py 24 0 > gpurun_out/r02_ld.txt 2>&1 || exit 1
grep -q '"bitwise_vs_packet_sweeps": true' gpurun_out/r02_ld.txt || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -k "ilu or large or 216" --timeout 100 --timeout-method thread > gpurun_out/r02_t1.log 2>&1
tail -3 gpurun_out/r02_t1.log
timeout -k 10 120 python tools/line_diag.py 216 0,8 >> gpurun_out/r02_ld.txt 2>&1 && timeout -k 10 100 python tools/line_trace.py 216 100 0 >> gpurun_out/r02_ld.txt 2>&1
