#!/bin/bash
# GPU box A/B of config 5's CG (tools/bench_configs.py cg-thermal) over library
# variants: default plus build/<v>.so for each argument (tools/build_variant.sh)
set -o pipefail
mkdir -p gpurun_out/c5
for v in default "$@" default "$@"; do
  if [ $v = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  timeout -k 10 200 python -u tools/bench_configs.py cg-thermal --ref-iters 10 > gpurun_out/c5/$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5/$v.json')); print('$v', d['gpu']['ms_per_iter'], d['gpu']['residual'], d['parity_serial_vs_reference']['trace_bitwise'])"
done
