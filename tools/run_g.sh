set -o pipefail
bash tools/gpu_exp.sh 216 x0 > gpurun_out/g_exp8.txt 2>&1 || { tail gpurun_out/g_exp8.txt; exit 1; }
bash tools/gpu_exp.sh 216 x0 >> gpurun_out/g_exp8.txt 2>&1 || { tail gpurun_out/g_exp8.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/g_exp8.txt
