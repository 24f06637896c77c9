# GPU box: U-sweep poller lead 2 on config 4's P = 8 slab (latency-bound) vs default (gpurun_out/g20/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g20; mkdir -p $O
for v in default dhu2 default dhu2; do
  if [ $v = default ]; then L=; else L=build/$v.so; fi
  echo "== $v"; LSSP_AMD_LIB=$L timeout -k 10 300 python -u tools/project_ranks.py --grid 512 --ranks 8 --steps 20 2>&1 | grep '^{' || exit 1
done | tee $O/p8_dhu2_ab.txt
