#!/bin/bash
# One GPU-box session, parametrised (replaces the per-session run_g*.sh /
# run_final_*.sh scripts of rounds 3-4):
#
#   tools/gpu_session.sh OUT step [step ...]
#
# Every step runs under its own time limit; the first failing step ends the
# session (no further GPU work after a fault, abort or timeout).  Outputs go
# to gpurun_out/OUT/.  Steps:
#   bench            python bench.py (headline + config4 + cpu_baseline) -> bench.json
#   prof             rocprofv3 --kernel-trace --stats of bench.py --steps 30 -> prof_bench/
#   pmc              two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) -> pmc_traffic.json
#   tests[=EXPR]     pytest -m gpu (optionally -k EXPR) -> pytest.log
#   file=PATH        pytest -m gpu on one test file -> pytest_<name>.log
#   quick=PATH       the same with a 120 s per-test limit and -x (new kernels)
#   project512       tools/project_ranks.py --grid 512 --ranks 1,8 -> project_ranks_512.jsonl
#   project216       tools/project_ranks.py --grid 216 --ranks 1,2,4,8 -> project_ranks_216.jsonl
#   prof5            rocprofv3 --kernel-trace of config 5 (CG) + tools/kgaps.py
#   config2 / config3 / config5 / general   tools/bench_configs.py bicgstab-iluk --grid 256 /
#                    gmres-ilut / cg-thermal / general-ilu
#   linediag=N[:LIB] tools/line_diag.py N 0 (optionally with LSSP_AMD_LIB=build/LIB.so)
#   linetrace=N      tools/line_trace.py N 150 -> line_trace_N.txt
#   pk6trace=N       tools/pk6_trace.py N 60 ilut -> pk6_trace_N.txt
#   serialdot        tools/serial_dot_probe.py -> serial_dot.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:?usage: gpu_session.sh OUT step ...}; shift
O=gpurun_out/$OUT; mkdir -p "$O"

fail() { echo "step '$1' failed (status $2)"; exit 1; }

for step in "$@"; do
  echo "== $step ($(date +%T))"
  case "$step" in
  bench)
    timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; fail $step $?; }
    python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline_spmv']['frac'], (d.get('config4') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
    ;;
  prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 30 --no-cpu --config4-steps 0 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; fail $step $?; }
    find $O/prof_bench -name "*kernel_stats.csv"
    ;;
  pmc)
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python3 bench.py --steps 10 --warmup 2 --no-cpu --config4-steps 0 > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; fail $step $?; }
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python3 bench.py --steps 10 --warmup 2 --no-cpu --config4-steps 0 > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; fail $step $?; }
    python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json || fail $step $?
    ;;
  tests|tests=*)
    K=${step#tests}; K=${K#=}
    timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; fail $step $?; }
    tail -3 $O/pytest.log
    ;;
  file=*)
    F=${step#file=}; B=$(basename "$F" .py)
    timeout -k 10 1200 python -u -m pytest "$F" -m gpu -v -s --timeout 900 --timeout-method thread > $O/pytest_$B.log 2>&1 || { tail -40 $O/pytest_$B.log; fail $step $?; }
    tail -3 $O/pytest_$B.log
    ;;
  quick=*)
    F=${step#quick=}; B=$(basename "$F" .py)
    timeout -k 10 400 python -u -m pytest "$F" -m gpu -v -s -x --timeout 120 --timeout-method thread > $O/pytest_$B.log 2>&1 || { tail -40 $O/pytest_$B.log; fail $step $?; }
    tail -3 $O/pytest_$B.log
    ;;
  project512)
    timeout -k 10 400 python -u tools/project_ranks.py --grid 512 --ranks 1,8 --steps 20 > $O/project_ranks_512.log 2>&1 || { tail -20 $O/project_ranks_512.log; fail $step $?; }
    grep '^{' $O/project_ranks_512.log | tee $O/project_ranks_512.jsonl
    ;;
  project216)
    timeout -k 10 300 python -u tools/project_ranks.py --grid 216 --ranks 1,2,4,8 > $O/project_ranks_216.log 2>&1 || { tail -20 $O/project_ranks_216.log; fail $step $?; }
    grep '^{' $O/project_ranks_216.log | tee $O/project_ranks_216.jsonl
    ;;
  config3)
    timeout -k 10 900 python -u tools/bench_configs.py gmres-ilut > $O/config3.json 2> $O/config3.err || { tail -20 $O/config3.err; fail $step $?; }
    tail -c 600 $O/config3.json
    ;;
  config2)
    timeout -k 10 600 python -u tools/bench_configs.py bicgstab-iluk --grid 256 > $O/config2.json 2> $O/config2.err || { tail -20 $O/config2.err; fail $step $?; }
    tail -c 900 $O/config2.json
    ;;
  prof5)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_config5 -o cg -- python3 tools/bench_configs.py cg-thermal --ref-iters 0 > $O/prof_config5.log 2>&1 || { tail -20 $O/prof_config5.log; fail $step $?; }
    python3 tools/kgaps.py $(find $O/prof_config5 -name "*kernel_trace.csv") --last 3000 | head -20
    ;;
  config5)
    timeout -k 10 300 python -u tools/bench_configs.py cg-thermal > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; fail $step $?; }
    tail -c 600 $O/config5.json
    ;;
  general)
    timeout -k 10 600 python -u tools/bench_configs.py general-ilu --ref-iters 0 > $O/general_ilu.jsonl 2> $O/general_ilu.err || { tail -20 $O/general_ilu.err; fail $step $?; }
    cut -c1-300 $O/general_ilu.jsonl
    ;;
  linediag=*)
    A=${step#linediag=}; N=${A%%:*}; LIB=; [ "$A" != "$N" ] && LIB=$PWD/build/${A#*:}.so
    LSSP_AMD_LIB=$LIB timeout -k 10 200 python -u tools/line_diag.py "$N" 0 2>&1 | grep -v amdgpu.ids | tee -a $O/line_diag.txt || fail $step $?
    ;;
  linetrace=*)
    N=${step#linetrace=}
    timeout -k 10 200 python -u tools/line_trace.py "$N" 150 2>&1 | grep -v amdgpu.ids > $O/line_trace_$N.txt || fail $step $?
    tail -30 $O/line_trace_$N.txt
    ;;
  pk6trace=*)
    N=${step#pk6trace=}
    timeout -k 10 300 python -u tools/pk6_trace.py "$N" 60 ilut 2>&1 | grep -v amdgpu.ids > $O/pk6_trace_$N.txt || fail $step $?
    tail -30 $O/pk6_trace_$N.txt
    ;;
  serialdot)
    timeout -k 10 200 python -u tools/serial_dot_probe.py > $O/serial_dot.txt 2>&1 || { tail -20 $O/serial_dot.txt; fail $step $?; }
    cat $O/serial_dot.txt
    ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
