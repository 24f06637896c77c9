set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py tests/test_gpu_integration.py -m gpu -x -q --timeout 600 --timeout-method thread -k "ilu or solver or trisolve or ilut or exam or driver" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/variant_ab.sh r06p 2 "python tools/apply_probe.py 128 ilut 10 && python tools/apply_probe.py 256 ilut 5" ext2 || exit 1
timeout -k 10 900 python -u tools/bench_configs.py gmres-ilut > $O/config3.json 2> $O/config3.err || { tail -20 $O/config3.err; exit 1; }
tail -c 1500 $O/config3.json
