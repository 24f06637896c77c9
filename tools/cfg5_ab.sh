set -o pipefail
mkdir -p gpurun_out
B="python -u tools/bench_configs.py cg-thermal --ref-iters 10"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest2.log 2>&1 || { tail -30 gpurun_out/gputest2.log; exit 1; }
tail -2 gpurun_out/gputest2.log
timeout -k 10 200 $B > gpurun_out/c5_fused2.json 2>/dev/null || exit 1
LSSP_AMD_CG_FUSE_L2=0 timeout -k 10 200 $B > gpurun_out/c5_unfused.json 2>/dev/null || exit 1
LSSP_AMD_LIB=$PWD/build/cgf1.so timeout -k 10 200 $B > gpurun_out/c5_fused1.json 2>/dev/null || exit 1
LSSP_AMD_LIB=$PWD/build/cgf4.so timeout -k 10 200 $B > gpurun_out/c5_fused4.json 2>/dev/null || exit 1
for f in fused2 unfused fused1 fused4; do python -c "import json,sys; d=json.load(open('gpurun_out/c5_$f.json')); print('$f', d['gpu'], d['spmv']['ms'])"; done
