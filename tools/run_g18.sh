# GPU box: non-temporal stores of the rhs gather / the L sweep's U-stream writes (gpurun_out/g18/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g18; mkdir -p $O
for v in default rhsnt out2nt bothnt default rhsnt out2nt bothnt; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 216"; LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep '^{' || exit 1
done | tee $O/nt_store_ab.txt
for v in default bothnt default bothnt; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 512"; LSSP_AMD_LIB=$L LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep '^{' || exit 1
done | tee -a $O/nt_store_ab.txt
