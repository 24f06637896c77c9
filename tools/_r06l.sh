set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ilu or solver or trisolve" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/variant_ab.sh r06l 2 "python tools/apply_probe.py 128 ilut 10 && python tools/apply_probe.py 256 ilut 5" gate0 gate2 || exit 1
timeout -k 10 300 python -u tools/pk6_trace.py 256 60 ilut > $O/pk6_trace_256.txt 2>&1 || { tail $O/pk6_trace_256.txt; exit 1; }
grep -v amdgpu.ids $O/pk6_trace_256.txt
