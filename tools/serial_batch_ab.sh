set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sb
for v in base sb32 sb64 base; do
  L=; [ $v != base ] && L=$PWD/build/$v.so
  LSSP_AMD_LIB=$L timeout -k 10 120 python -u tools/serial_dot_probe.py > gpurun_out/sb/$v.txt 2>&1 || exit 1
  echo "$v $(grep '^{' gpurun_out/sb/$v.txt | tr '\n' ' ')"
done
