# GPU box: probe + full GPU suite + bench line + rocprofv3 kernel stats (gpurun_out/g1/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 60 tools/probe/shfl_probe > $O/shfl_probe.txt 2>&1; cat $O/shfl_probe.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -s > $O/pytest.log 2>&1
tail -3 $O/pytest.log; grep -E "^(bicgstab|gmres|512)" $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
