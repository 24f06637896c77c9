# GPU box: non-temporal coefficient stream (rhs temporal) vs both nt vs default: apply and bench (gpurun_out/g17/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g17; mkdir -p $O
for v in default coefnt dmant default coefnt dmant; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 216"; LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep '^{' || exit 1
  echo "== $v 512"; LSSP_AMD_LIB=$L LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep '^{' || exit 1
done | tee $O/nt_ab.txt
for v in default coefnt dmant; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  LSSP_AMD_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['ms_per_launch'])"
done | tee -a $O/nt_ab.txt
