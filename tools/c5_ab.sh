#!/bin/bash
# Interleaved A/B of library builds on the C5 adversarial config (exp_libs/lib_*.so via BLSMI355X_LIB).
# Usage (via gpurun): bash tools/c5_ab.sh ROUNDS variant...
set -o pipefail
OUT=gpurun_out/c5ab; mkdir -p $OUT; export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=$PWD/exp_libs/lib_$v.so; [ "$v" = cur ] && lib=$PWD/eth-consensus-specs_amd/libblsmi355x.so
    BLSMI355X_LIB=$lib timeout -k 10 120 python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu --no-percall \
      --no-parity --no-profile > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { echo "$v FAILED"; tail -3 $OUT/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json')); print('$v', d['value'], d['ms_per_step'], d['fallback_last_step'])"
  done
done
