#!/bin/bash
# rocprofv3 counter passes over a short bench run, one pass per counter group
# (FETCH_SIZE for HBM bytes; SQ issue/wait counters).  Usage (via gpurun): bash tools/pmc_pass.sh TAG
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-profile --no-percall --c4-steps 0 --c5-steps 0 --no-regload > "$OUT/fetch.log" 2>&1 || { tail -20 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  --output-format csv -d "$OUT/sq" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-profile --no-percall --c4-steps 0 --c5-steps 0 --no-regload > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/lds" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-profile --no-percall --c4-steps 0 --c5-steps 0 --no-regload > "$OUT/lds.log" 2>&1 || { tail -20 "$OUT/lds.log"; exit 1; }
for p in fetch sq lds; do
  f=$(find "$OUT/$p" -name '*counter_collection.csv' | head -n 1)
  [ -n "$f" ] && python3 tools/pmc_summary.py "$f" "$OUT/pmc_$p.md" > /dev/null
done
ls "$OUT"
