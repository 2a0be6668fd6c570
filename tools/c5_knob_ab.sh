#!/bin/bash
# Interleaved A/B of env knobs on the C5 adversarial config.  Usage (via gpurun): bash tools/c5_knob_ab.sh ROUNDS "VAR=V ..." ...
set -o pipefail
OUT=gpurun_out/c5kab; mkdir -p $OUT; export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for kv in "$@"; do
    i=$((i+1)); envs=""; [ "$kv" != base ] && envs="$kv"
    env $envs timeout -k 10 120 python3 bench.py --config c5 --steps 30 --warmup 3 --no-cpu --no-percall \
      --no-parity --no-profile > $OUT/k$i.$r.json 2> $OUT/k$i.$r.err || { echo "[$kv] FAILED"; tail -3 $OUT/k$i.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k$i.$r.json')); print('[$kv]', d['value'], d['ms_per_step'], d['fallback_last_step'])"
  done
done
