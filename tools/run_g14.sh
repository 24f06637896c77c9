# GPU box: k_line2 poller / loader leads per sweep after the per-lane masks (gpurun_out/g14/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g14; mkdir -p $O
for v in default dhu2 dh2 dhu2d5 nosleep default dhu2 dh2 dhu2d5 nosleep; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 216"; LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep '^{' || exit 1
done | tee $O/leads_ab.txt
for v in default dhu2 default dhu2; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 512"; LSSP_AMD_LIB=$L LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep '^{' || exit 1
done | tee -a $O/leads_ab.txt
