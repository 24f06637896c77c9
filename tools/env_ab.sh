#!/bin/bash
# Tuning aid (GPU box): a command under several environment settings,
# alternated -- tools/env_ab.sh OUT REPS "CMD" "ENV1" "ENV2" ...  ("-" = none)
set -o pipefail
O=gpurun_out/$1; REPS=$2; CMD=$3; shift 3; mkdir -p $O
for rep in $(seq $REPS); do for e in "$@"; do
  echo "== $e" >> $O/ab.txt
  if [ "$e" = "-" ]; then timeout -k 10 300 bash -c "$CMD" >> $O/ab.txt 2>>$O/err.txt || exit 1
  else env $e timeout -k 10 300 bash -c "$CMD" >> $O/ab.txt 2>>$O/err.txt || exit 1; fi
done; done
