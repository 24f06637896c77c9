# GPU box: windowed SpMV pipelining + CG prologue (config 5) -- parity, then A/B (gpurun_out/g11/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k config5 tests/test_gpu_parity.py -k "scattered or sliced or config5" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for v in pipe0 default nk9 nk10 pipe0 default; do
  case $v in pipe0) E="LSSP_AMD_SELL_PIPE=0"; L=;; default) E=; L=;; nk9) E=; L=build/sell_nk9.so;; nk10) E=; L=build/sell_nk10.so;; esac
  echo "== $v"
  env $E LSSP_AMD_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py cg-thermal --iters 1000 --ref-iters 30 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'spmv_ms': d['spmv']['ms'], 'spmv_GBps': d['spmv']['GBps'], 'cg_us_per_it': round(d['gpu']['ms_per_iter']*1e3,2), 'residual': d['gpu']['residual'], 'serial30_bitwise': d.get('parity_serial_vs_reference', {}).get('trace_bitwise')}))" || exit 1
done | tee $O/ab.txt
