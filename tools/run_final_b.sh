# GPU box: measurement set B -- config 4 on one GPU, 8-GPU projections, configs 3 and 5, k_line vs k_line2 at 512^3 (gpurun_out/fb/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/fb; mkdir -p $O
timeout -k 10 300 python -u tools/project_ranks.py --grid 216 --ranks 1,2,4,8 2>&1 | grep -v amdgpu | tee $O/project_ranks_216.jsonl
timeout -k 10 400 python -u tools/project_ranks.py --grid 512 --ranks 1,8 --steps 20 2>&1 | grep -v amdgpu | tee $O/project_ranks_512.jsonl
for N in 216 512; do for v in diag row diag row; do echo "== ${N}^3 claim order $v"; LSSP_AMD_LINE2_ROWORDER=$([ $v = row ] && echo 1 || echo 0) LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py $N 0 2>&1 | grep -v amdgpu; done; done | tee $O/claim_order.txt
for m in 2 1; do echo "== 512^3 LSSP_AMD_LINE_MODE=$m"; LSSP_AMD_LINE_MODE=$m LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep -v amdgpu; done | tee $O/line_mode_512.txt
timeout -k 10 500 python -u tools/bench_configs.py bicgstab-iluk --grid 512 > $O/config4_512.json 2> $O/config4_512.err; tail -c 600 $O/config4_512.json
timeout -k 10 300 python -u tools/bench_configs.py cg-thermal > $O/config5.json 2> $O/config5.err; tail -c 600 $O/config5.json
