# GPU box: per-step trace of the final k_line2 at 216^3 (gpurun_out/g19/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 300 python -u tools/line_trace.py 216 2>&1 | grep -v amdgpu | tee $O/line_trace.txt
