# GPU box: ILU(1) line sweeps -- kernel stats at 128^3 and timing variants (gpurun_out/g10/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g10; mkdir -p $O
LINE_DIAG_LEVEL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 tools/line_diag.py 128 0 > $O/prof.txt 2>&1 || exit 1
grep '^{' $O/prof.txt
for v in default f_n4 f_nodiv f_dh2 f_d5; do
  echo "== $v"
  if [ $v = default ]; then LIB=; else LIB=build/$v.so; fi
  LSSP_AMD_LIB=$LIB LINE_DIAG_LEVEL=1 LINE_DIAG_NOCHECK=1 timeout -k 10 200 python3 tools/line_diag.py 128 0 2>&1 | grep '^{' || exit 1
done | tee $O/variants.txt
