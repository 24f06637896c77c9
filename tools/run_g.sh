set -o pipefail
O=gpurun_out/ab; mkdir -p $O
for v in default nofuse default nofuse; do
  if [ "$v" = default ]; then unset LSSP_AMD_LIB; else export LSSP_AMD_LIB=$PWD/build/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
