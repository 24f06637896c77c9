# GPU box: closing verification of the round's final code -- bench line, kernel stats, HBM PMC,
# GPU suite, config 4's rank projection (gpurun_out/fe2/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/fe2; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline_spmv']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 30 --no-cpu > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u tools/project_ranks.py --grid 512 --ranks 1,8 --steps 20 2>&1 | grep '^{' | tee $O/project_ranks_512.jsonl
