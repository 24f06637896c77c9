#!/bin/bash
# GPU box: the round's evidence -- bench line, rocprofv3 kernel stats of the
# bench and of config 5's CG, config 5 with full-size parity.  Outputs under
# gpurun_out/ev/ (copied into profiles/ afterwards).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ev; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o bench -- python3 bench.py --steps 30 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cg -o cg -- python3 tools/bench_configs.py cg-thermal --ref-iters 10 > $O/prof_cg.log 2>&1 || { tail -20 $O/prof_cg.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py cg-thermal > $O/config5_cg.json 2> $O/config5_cg.err || { tail -20 $O/config5_cg.err; exit 1; }
for d in prof_bench prof_cg; do
  db=$(find $O/$d -name "*results.db" | head -1)
  [ -n "$db" ] && timeout -k 10 120 rocpd2summary -i "$db" -d $O/$d/summary --format csv > /dev/null 2>&1
done
find $O -name "*summary.csv" | sort
tail -c 400 $O/bench.json; tail -c 600 $O/config5_cg.json
