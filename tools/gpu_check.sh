#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh TAG [tests|bench|prof]...
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
TAG=${1:-run}
shift
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
      tail -3 "$OUT/pytest.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    benchq)
      timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    prof)
      (cd /tmp && true)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1 \
        || { tail -30 "$OUT/prof.log"; exit 1; }
      db=$(find "$OUT/prof" -name '*.db' | head -n 1)
      if [ -n "$db" ]; then python3 tools/rocprof_summary.py "$db" "$OUT/kernel_stats.md" > /dev/null; fi
      find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
      tail -2 "$OUT/prof.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
