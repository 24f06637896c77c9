set -o pipefail
bash tools/gpu_exp.sh 216 ls3 ls0 nl5 nl3 > gpurun_out/g_exp5.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/g_exp5.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile_shapes or trisolve_sweeps or ilu" --timeout 120 --timeout-method thread > gpurun_out/g_pt.log 2>&1
tail -2 gpurun_out/g_pt.log
