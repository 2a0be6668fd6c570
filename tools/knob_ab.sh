#!/bin/bash
# A/B of env knobs: each argument is a space-separated "VAR=VALUE ..." set (or "base").  The sets run
# interleaved REPS times (default 3), STEPS timed passes each (default 60); the median per set is printed.
# Usage (via gpurun): REPS=3 bash tools/knob_ab.sh TAG "base" "BLS_FAV_JOBS_INIT=6" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
REPS=${REPS:-3}; STEPS=${STEPS:-60}
for r in $(seq 1 $REPS); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    envs=""; [ "$kv" != base ] && envs="$kv"
    env $envs timeout -k 10 150 python3 bench.py --steps $STEPS --warmup 3 --no-cpu --no-percall --no-e2e --roofline-passes 2 --c4-steps 0 --c5-steps 0 --no-regload \
      > $OUT/k${i}_r$r.json 2> $OUT/k${i}_r$r.err || { echo "[$kv] FAILED rc=$?"; tail -3 $OUT/k${i}_r$r.err | cut -c1-300; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k${i}_r$r.json')); print('[$kv] r$r', d['value'], (d.get('c3') or {}).get('fav_s'), 'frac', d['roofline']['frac'], 'launch_ms', d['roofline']['avg_launch_ms'])"
  done
done
i=0
for kv in "$@"; do
  i=$((i+1))
  python3 - "$OUT" "$i" "$kv" <<'PY'
import glob, json, statistics, sys
out, i, kv = sys.argv[1:]
ds = [json.load(open(f)) for f in glob.glob(f"{out}/k{i}_r*.json")]
v = sorted(d["value"] for d in ds)
c3 = sorted((d.get("c3") or {}).get("fav_s") or 0 for d in ds)
print(f"[{kv}] median C2 {statistics.median(v):.0f} C3 {statistics.median(c3):.0f}  all {[round(x) for x in v]} {[round(x) for x in c3]}")
PY
done
