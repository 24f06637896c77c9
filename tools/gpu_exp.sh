export LSSP_AMD_LINE_M=1
for v in default dh2; do
  if [ $v = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/line_diag.py 216 0,0 || exit 1
done
