#!/bin/bash
# Tuning aid (GPU box): one command under the in-tree library and variant
# builds (tools/build_variant.sh -> build/<name>.so, loaded via LSSP_AMD_LIB),
# alternated REPS times in one session (boxes differ by ~2 %, so A/B runs stay
# inside one call):
#   tools/variant_ab.sh OUT REPS "CMD" name ...
# CMD defaults to the 216^3 bench ("python bench.py --steps 100 --no-cpu
# --config4-steps 0"); e.g. "python tools/project_ranks.py --grid 512 --ranks 8",
# "python tools/pk6_trace.py 128 60 ilut", "python tools/tail_bench.py".
set -o pipefail
O=gpurun_out/$1; REPS=${2:-3}; CMD=${3:-python bench.py --steps 100 --warmup 10 --no-cpu --config4-steps 0}
shift 3; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in $(seq $REPS); do
  for v in default "$@"; do
    echo "== $v" >> $O/ab.txt
    if [ $v = default ]; then L=; else L=$R/build/$v.so; fi
    LSSP_AMD_LIB=$L timeout -k 10 300 bash -c "$CMD" >> $O/ab.txt 2>>$O/err.txt || exit 1
  done
done
