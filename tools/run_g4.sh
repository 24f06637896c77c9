# GPU box: k_line2 Markstein / lead variants + bench + trace (gpurun_out/g4/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "tile_shapes or ilu" > $O/parity.log 2>&1; tail -2 $O/parity.log
export LINE_DIAG_NOCHECK=1
for v in default m_dh2 m_nodiv m_nodiv_dh2 m_dh2_d5 m_dh2_d8 default m_dh2; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/line_diag.py 216 0 || { echo "variant $v failed"; exit 1; }
done 2>&1 | grep -v amdgpu.ids | tee $O/variants.txt
unset LSSP_AMD_LIB LINE_DIAG_NOCHECK
timeout -k 10 120 python -u tools/line_trace.py 216 150 > $O/line_trace.txt 2>&1; cat $O/line_trace.txt | grep -v amdgpu
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline_spmv']['frac'], d['roofline']['peak_measured_detail'])"
