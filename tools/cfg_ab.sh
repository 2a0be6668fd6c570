#!/bin/bash
# A/B of env knobs on one bench config: CFG=c3|c5|c2 REPS=n bash tools/cfg_ab.sh TAG "base" "VAR=VALUE ..." ...
# interleaved runs of `bench.py --config $CFG`; prints each run's value and the median per arm.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
REPS=${REPS:-3}; STEPS=${STEPS:-60}; CFG=${CFG:-c3}
for r in $(seq 1 $REPS); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    envs=""; [ "$kv" != base ] && envs="$kv"
    env $envs timeout -k 10 200 python3 bench.py --config $CFG --steps $STEPS --warmup 3 --no-cpu --no-percall --no-e2e \
      --no-parity --roofline-passes 2 --no-regload > $OUT/k${i}_r$r.json 2> $OUT/k${i}_r$r.err \
      || { echo "[$kv] FAILED rc=$?"; tail -3 $OUT/k${i}_r$r.err | cut -c1-300; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k${i}_r$r.json')); print('[$kv] r$r', d['value'])"
  done
done
i=0
for kv in "$@"; do
  i=$((i+1))
  python3 - "$OUT" "$i" "$kv" <<'PY'
import glob, json, statistics, sys
out, i, kv = sys.argv[1:]
v = sorted(json.load(open(f))["value"] for f in glob.glob(f"{out}/k{i}_r*.json"))
print(f"[{kv}] median {statistics.median(v):.0f}  all {[round(x) for x in v]}")
PY
done
