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
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
      tail -3 "$OUT/pytest.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    configs)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread \
        > "$OUT/configs.log" 2>&1 || { tail -40 "$OUT/configs.log"; exit 1; }
      tail -3 "$OUT/configs.log" ;;
    benchq)
      timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    prof)
      (cd /tmp && true)
      # the bench command itself (the CPU leg is host-only and skipped under the profiler)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
        python3 bench.py --no-cpu > "$OUT/prof.log" 2>&1 \
        || { tail -30 "$OUT/prof.log"; exit 1; }
      db=$(find "$OUT/prof" -name '*.db' | head -n 1)
      if [ -n "$db" ]; then python3 tools/rocprof_summary.py "$db" "$OUT/kernel_stats.md" "$OUT/rocprof_kernel_avg.json" \
        "profiles/${TAG}_kernel_stats.md (rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu)" > /dev/null; fi
      find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
      tail -2 "$OUT/prof.log" ;;
    profc2)
      # C2 only, one batch at a time (--no-pipeline): the per-(kernel, grid) averages bench.py's frac_rocprof reads
      # (profiles/rocprof_kernel_avg.json), comparable with its one-batch-at-a-time hipEvent figure
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/profc2" -o run -- \
        python3 bench.py --no-cpu --no-pipeline --steps 20 --c3-steps 0 --c4-steps 0 --c5-steps 0 --no-percall \
        --no-parity --no-e2e > "$OUT/profc2.log" 2>&1 || { tail -30 "$OUT/profc2.log"; exit 1; }
      db=$(find "$OUT/profc2" -name '*.db' | head -n 1)
      if [ -n "$db" ]; then python3 tools/rocprof_summary.py "$db" "$OUT/c2_kernel_stats.md" "$OUT/rocprof_kernel_avg.json" \
        "profiles/${TAG}_c2_kernel_stats.md (rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --no-pipeline --steps 20 --c3-steps 0 --c4-steps 0 --c5-steps 0 --no-percall --no-parity --no-e2e)" > /dev/null; fi
      tail -1 "$OUT/profc2.log" | cut -c1-300 ;;
    percall)
      timeout -k 10 120 python3 tools/percall_probe.py > "$OUT/percall.json" 2> "$OUT/percall.err" \
        || { tail -20 "$OUT/percall.err"; exit 1; }
      cat "$OUT/percall.json"
      REPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pcprof" -o run -- \
        python3 tools/percall_probe.py > "$OUT/pcprof.log" 2>&1 || { tail -20 "$OUT/pcprof.log"; exit 1; }
      db=$(find "$OUT/pcprof" -name '*.db' | head -n 1)
      if [ -n "$db" ]; then python3 tools/rocprof_summary.py "$db" "$OUT/percall_kernel_stats.md" "$OUT/percall_avg.json" \
        "profiles/${TAG}_percall_kernel_stats.md (rocprofv3 --kernel-trace --stats -- python3 tools/percall_probe.py)" > /dev/null; fi
      find "$OUT/pcprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/percall_kernel_stats.csv" \; ;;
    c3tl)
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/c3tl" -o run -- \
        python3 bench.py --config c3 --steps 25 --warmup 2 --no-cpu --no-percall --no-parity --no-e2e --no-profile \
        > "$OUT/c3tl.log" 2>&1 || { tail -20 "$OUT/c3tl.log"; exit 1; }
      tail -1 "$OUT/c3tl.log"
      db=$(find "$OUT/c3tl" -name '*.db' | head -n 1)
      if [ -n "$db" ]; then python3 tools/timeline.py "$db" k_miller_acc4 2 24 > "$OUT/c3_timeline.txt" 2>&1 || true; head -12 "$OUT/c3_timeline.txt"; fi ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
