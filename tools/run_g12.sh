# GPU box: k_line2 with four levels per step -- parity, then A/B against two (gpurun_out/g12/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g12; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "tile_shapes or trisolve_sweeps" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for N in 216 512; do for lv in 2 4 2 4; do echo "== ${N}^3 LV=$lv"; LSSP_AMD_LINE_LV=$lv LINE_DIAG_NOCHECK=1 timeout -k 10 200 python tools/line_diag.py $N 0 2>&1 | grep '^{' || exit 1; done; done | tee $O/lv_ab.txt
for lv in 4 2; do LSSP_AMD_LINE_LV=$lv timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_lv$lv.json 2> $O/bench_lv$lv.err || exit 1; python3 -c "import json; d=json.load(open('$O/bench_lv$lv.json')); print('LV=$lv', d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"; done
