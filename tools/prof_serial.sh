# standalone per-kernel work: one stream, one batch in flight, under rocprofv3
set -o pipefail
OUT=gpurun_out/${1:-ser}
mkdir -p $OUT
export TMPDIR=/tmp
BLS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-pipeline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
db=$(find $OUT/prof -name '*.db' | head -n 1)
python3 tools/rocprof_summary.py "$db" $OUT/kernel_stats.md > /dev/null
grep -v "^W2" $OUT/prof.log | tail -1 | cut -c1-200
