#!/bin/bash
# C2 pipeline timeline per env variant: rocprofv3 --kernel-trace over a short C2 bench run, then tools/timeline.py
# (per-kernel in-pipeline durations and wave-ms per batch).  Usage (via gpurun): bash tools/c2_timeline.sh TAG "ENV..." ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for kv in "$@"; do
  i=$((i+1))
  envs=""; [ "$kv" != base ] && envs="$kv"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/t$i" -o run -- \
    python3 bench.py --steps 30 --warmup 2 --no-cpu --no-percall --no-parity --no-e2e --no-profile --no-regload \
    --c3-steps 0 --c4-steps 0 --c5-steps 0 > "$OUT/t$i.log" 2>&1 || { echo "[$kv] FAILED"; tail -5 "$OUT/t$i.log"; exit 1; }
  db=$(find "$OUT/t$i" -name '*.db' | head -n 1)
  echo "== [$kv] $(python3 -c "import json,sys; d=json.loads(open('$OUT/t$i.log').read().strip().splitlines()[-1]); print(d['value'])")"
  python3 tools/timeline.py "$db" k_miller_acc4 4 24 > "$OUT/timeline_$i.txt" 2>&1; head -14 "$OUT/timeline_$i.txt"
  rm -rf "$OUT/t$i"
done
