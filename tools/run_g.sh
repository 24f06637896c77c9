# GPU box: the round's verification -- full GPU suite, bench line, rocprofv3
# kernel stats of the bench (outputs under gpurun_out/final/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 30 --no-cpu > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
find $O -name "*kernel_stats.csv"
