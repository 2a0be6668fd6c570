#!/bin/bash
# A/B of library builds (exp_libs/lib_*.so via BLSMI355X_LIB): one-batch kernel times + throughput.
set -o pipefail
OUT=gpurun_out/libab; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/exp_libs/lib_$v.so; [ "$v" = cur ] && lib=$PWD/eth-consensus-specs_amd/libblsmi355x.so
  BLSMI355X_LIB=$lib timeout -k 10 150 python3 bench.py --steps 40 --warmup 3 --no-cpu --no-percall --no-e2e \
    > $OUT/$v.json 2> $OUT/$v.err || { echo "$v FAILED"; tail -3 $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); k=d['kernels_avg_ms']; print('$v', d['value'], 'miller', k['miller'], 'sig_vm', k['sig_vm'], 'hash', k['fav_hash'], 'msm', k['msm'], 'fe', k['final_exp'], 'frac', d['roofline']['frac'], 'c3', (d.get('c3') or {}).get('fav_s'))"
done
