set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/fe_probe.py 40 > $OUT/probe.log 2>&1 && cat $OUT/probe.log &&
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 tools/fe_probe.py 20 > $OUT/kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 tools/fe_probe.py 10 > $OUT/sq.log 2>&1 &&
f=$(find $OUT/sq -name '*counter_collection.csv' | head -n 1) && python3 tools/pmc_summary.py "$f" $OUT/pmc_sq.md | grep -E "fe_check|kernel" ;
find $OUT/kt -name '*kernel_stats.csv' -exec grep -h "fe_check" {} \;
