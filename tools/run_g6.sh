# GPU box: stream reciprocals (NA 5) vs IEEE division, parity subset, bench (gpurun_out/g6/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_refconv.py -q -x --timeout 300 --timeout-method thread -k "tile_shapes or ilu or 512 or refconv or bicgstab" > $O/parity.log 2>&1; tail -2 $O/parity.log
for r in 1 0 1 0; do echo "== LSSP_AMD_LINE2_RCP=$r"; LSSP_AMD_LINE2_RCP=$r timeout -k 10 120 python tools/line_diag.py 216 0 2>&1 | grep -v amdgpu; done | tee $O/rcp_ab.txt
timeout -k 10 120 python -u tools/line_trace.py 216 150 2>&1 | grep -v amdgpu > $O/line_trace.txt; cat $O/line_trace.txt
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
for P in 8 16; do echo "== 512^3 P=$P"; LSSP_AMD_LINE2_P=$P LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py 512 0 2>&1 | grep -v amdgpu; done | tee $O/p_512.txt
