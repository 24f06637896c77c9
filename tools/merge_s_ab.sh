set -o pipefail
mkdir -p gpurun_out/ms
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ms/gputest.log 2>&1 || { tail -40 gpurun_out/ms/gputest.log; exit 1; }
tail -1 gpurun_out/ms/gputest.log
for v in merged unmerged merged unmerged; do
  if [ $v = unmerged ]; then export LSSP_AMD_BICG_MERGE_S=0; else unset LSSP_AMD_BICG_MERGE_S; fi
  timeout -k 10 120 python -u bench.py --no-cpu --steps 200 > gpurun_out/ms/$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ms/$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
