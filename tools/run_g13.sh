# GPU box: compute-wave variants of k_line2 (lane-16 shuffle by permlane swaps; j/i products
# formed before the k shuffle; row masks by per-lane compares) vs default (gpurun_out/g13/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g13; mkdir -p $O
for v in default permlane hoist vmask hoistvm default permlane hoist vmask hoistvm; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v ILU(0) 216"; LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep '^{' || exit 1
done | tee $O/variants_ab.txt
for v in default permlane default permlane; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v ILU(1) 128"; LSSP_AMD_LIB=$L LINE_DIAG_LEVEL=1 timeout -k 10 200 python tools/line_diag.py 128 0 2>&1 | grep '^{' || exit 1
done | tee -a $O/variants_ab.txt
