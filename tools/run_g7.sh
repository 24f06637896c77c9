# GPU box: kernel stats of the 8-rank projection's rank-0 slab (512^3 and 216^3) (gpurun_out/g7/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g7; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p512 -o run -- python3 tools/project_ranks.py --grid 512 --ranks 8 --steps 20 > $O/p512.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p216 -o run -- python3 tools/project_ranks.py --grid 216 --ranks 8 --steps 30 > $O/p216.txt 2>&1
rc=$?; grep '^{' $O/p512.txt $O/p216.txt; find $O -name '*kernel_stats.csv' | head; exit $rc
