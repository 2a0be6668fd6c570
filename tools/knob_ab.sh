#!/bin/bash
# A/B of env knobs: each argument is a space-separated "VAR=VALUE ..." set (or "base"), one 40-step bench each.
# Usage (via gpurun): bash tools/knob_ab.sh TAG "base" "BLS_XC_G=1" "BLS_XC_G=1 BLS_FAV_JOBS_INIT=6" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for kv in "$@"; do
  i=$((i+1))
  envs=""; [ "$kv" != base ] && envs="$kv"
  env $envs timeout -k 10 150 python3 bench.py --steps 40 --warmup 3 --no-cpu --no-percall --no-e2e \
    > $OUT/k$i.json 2> $OUT/k$i.err || { echo "[$kv] FAILED rc=$?"; tail -3 $OUT/k$i.err | cut -c1-300; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/k$i.json')); k=d['kernels_avg_ms']; print('[$kv]', d['value'], 'miller', k['miller'], 'hash', k['fav_hash'], 'frac', d['roofline']['frac'])"
done
