set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ev; mkdir -p $O
bash tools/gpu_exp.sh 216 ls3 ls0 nl5 nl3 drn > $O/exp5.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/exp5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o bench -- python3 bench.py --steps 30 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -k 10 400 python -u tools/bench_configs.py cg-thermal > $O/config5_cg.json 2> $O/config5_cg.err || { tail -5 $O/config5_cg.err; exit 1; }
tail -c 300 $O/config5_cg.json
