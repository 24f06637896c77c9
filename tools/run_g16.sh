# GPU box: non-temporal sweep streams A/B; config 3 (GMRES(30) + ILUT at 256^3) re-measured (gpurun_out/g16/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g16; mkdir -p $O
for v in default dmant default dmant; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v 216"; LSSP_AMD_LIB=$L timeout -k 10 200 python tools/line_diag.py 216 0 2>&1 | grep '^{' || exit 1
  echo "== $v 512"; LSSP_AMD_LIB=$L LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep '^{' || exit 1
done | tee $O/dmant_ab.txt
timeout -k 10 600 python -u tools/bench_configs.py gmres-ilut > $O/config3.json 2> $O/config3.err; tail -c 900 $O/config3.json
