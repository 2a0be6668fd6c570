#!/bin/bash
# SQ counters of one bench run with an env setting: bash tools/pmc_sq_env.sh TAG "VAR=VALUE ..." (or "base")
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp
envs=""; [ "$2" != base ] && envs="$2"
for kv in $envs; do export "$kv"; done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  --output-format csv -d "$OUT/sq" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-profile --no-percall --c4-steps 0 --c5-steps 0 --c3-steps 0 --no-regload --no-parity > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
f=$(find "$OUT/sq" -name '*counter_collection.csv' | head -n 1)
python3 tools/pmc_summary.py "$f" "$OUT/pmc_sq.md" > /dev/null
grep -i "miller_acc\|kernel" $OUT/pmc_sq.md | head -8
