#!/bin/bash
# C5 (adversarial 1,024 x 512, bisection every pass): kernel timeline + SQ wave residency per kernel.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tl" -o run -- \
  python3 bench.py --config c5 --steps 30 --warmup 2 --no-cpu --no-percall --no-parity --no-e2e --no-profile \
  > "$OUT/tl.log" 2>&1 || { tail -5 "$OUT/tl.log"; exit 1; }
db=$(find "$OUT/tl" -name '*.db' | head -n 1)
python3 tools/timeline.py "$db" k_miller_acc4 4 24 > "$OUT/c5_timeline.txt" 2>&1; head -30 "$OUT/c5_timeline.txt"
rm -rf "$OUT/tl"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  --output-format csv -d "$OUT/sq" -o run -- \
  python3 bench.py --config c5 --steps 6 --warmup 1 --no-cpu --no-percall --no-parity --no-e2e --no-profile > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
f=$(find "$OUT/sq" -name '*counter_collection.csv' | head -n 1)
cp "$f" "$OUT/sq.csv"
python3 tools/pmc_summary.py "$f" "$OUT/pmc_sq.md" > /dev/null
rm -rf "$OUT/sq"
