# GPU box: bench, kernel stats, full GPU suite, then k_line2 variants incl. scalar polls (gpurun_out/g5/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g5; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline_spmv']['frac'], d['roofline']['peak_measured_detail'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 30 --no-cpu > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -k 10 120 python -u tools/line_trace.py 216 150 2>&1 | grep -v amdgpu > $O/line_trace.txt; cat $O/line_trace.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
tail -4 $O/pytest.log
export LINE_DIAG_NOCHECK=1
for v in default v_d5 v_d4 v_dh2_d5 v_nl3 v_div2 v_ls6 v_ls3d4 default v_spoll v_spoll_d5; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/line_diag.py 216 0 || { echo "variant $v failed"; exit 1; }
done 2>&1 | grep -v amdgpu.ids | tee $O/variants.txt
unset LINE_DIAG_NOCHECK
unset LSSP_AMD_LIB
export LSSP_AMD_LINE2_P=16
echo "== P16 (default lib)"; timeout -k 10 120 python -u tools/line_diag.py 216 0 2>&1 | grep -v amdgpu | tee $O/check_p16.txt
export LSSP_AMD_LIB=$PWD/build/v_p16d5.so
echo "== P16 D5"; timeout -k 10 120 python -u tools/line_diag.py 216 0 2>&1 | grep -v amdgpu | tee $O/check_p16d5.txt
unset LSSP_AMD_LIB LSSP_AMD_LINE2_P
for v in v_div2 v_spoll; do export LSSP_AMD_LIB=$PWD/build/$v.so
timeout -k 10 120 python -u tools/line_diag.py 216 0 2>&1 | grep -v amdgpu | tee $O/check_$v.txt; done
export LSSP_AMD_LIB=$PWD/build/v_spoll.so
timeout -k 10 120 python -u tools/line_trace.py 216 150 2>&1 | grep -v amdgpu > $O/line_trace_spoll.txt; cat $O/line_trace_spoll.txt
