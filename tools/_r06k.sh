set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 200 python -u tools/pk6_trace.py 128 60 ilut > $O/pk6_trace_128.txt 2>&1 || { tail $O/pk6_trace_128.txt; exit 1; }
cat $O/pk6_trace_128.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/pk6_trace.py 256 60 ilut > $O/pk6_trace_256.txt 2>&1 || { tail $O/pk6_trace_256.txt; exit 1; }
cat $O/pk6_trace_256.txt | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o f -- python3 $GRAFT_REPO_ROOT/tools/apply_probe.py 256 ilut 5 > $GRAFT_REPO_ROOT/$O/pmc_fetch.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o w -- python3 $GRAFT_REPO_ROOT/tools/apply_probe.py 256 ilut 5 > $GRAFT_REPO_ROOT/$O/pmc_write.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_write.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 $GRAFT_REPO_ROOT/tools/apply_probe.py 256 ilut 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
