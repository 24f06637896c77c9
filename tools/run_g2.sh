# GPU box: k_line2 bring-up -- tile-shape parity, full GPU suite, bench, line trace, read probe (gpurun_out/g2/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 60 --timeout-method thread -k "tile_shapes" > $O/shapes.log 2>&1; rc=$?
tail -3 $O/shapes.log; [ $rc -eq 0 ] || { grep -E "^E|Error" $O/shapes.log | head -20; exit 1; }
timeout -k 10 60 tools/probe/read_probe > $O/read_probe.txt 2>&1; cat $O/read_probe.txt
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['roofline']['ms_per_launch'], d['roofline']['frac'])"
timeout -k 10 120 python -u tools/line_trace.py 216 150 > $O/line_trace.txt 2>&1; cat $O/line_trace.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
tail -8 $O/pytest.log
