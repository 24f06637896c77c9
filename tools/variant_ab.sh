#!/bin/bash
# Tuning aid (GPU box): 216^3 bench it/s of the default library against
# variant builds (build/<name>.so), alternated, plus kernel stats of the
# default -- tools/variant_ab.sh OUT name ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for v in default "$@"; do
    echo "== $v" >> $O/ab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LSSP_AMD_LIB=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0 >> $O/ab.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o b -- python3 $R/bench.py --steps 30 --no-cpu --config4-steps 0 > $R/$O/prof.log 2>&1 || exit 1
