# GPU box: k_line2 lead / wave-count variants (apply us at 216^3), gpurun_out/g3/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x --timeout 200 --timeout-method thread -k "tile_shapes or ilu or 512" > $O/parity.log 2>&1; tail -3 $O/parity.log
export LINE_DIAG_NOCHECK=1
for v in default l2_dh2 l2_d4 l2_d8 l2_nl2 l2_sw2 l2_perm default; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/line_diag.py 216 0 || { echo "variant $v failed"; exit 1; }
done 2>&1 | grep -v amdgpu.ids | tee $O/variants.txt
unset LSSP_AMD_LIB LINE_DIAG_NOCHECK
timeout -k 10 400 python -u tools/bench_stream_order.py 216 2>&1 | grep -v amdgpu.ids | tee $O/stream_order.txt
