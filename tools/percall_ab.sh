#!/bin/bash
# Interleaved per-call latency A/B of library builds (exp_libs/lib_*.so; "cur" = the in-tree library).
# Usage (via gpurun): bash tools/percall_ab.sh TAG lib1 lib2 ...   (each list is run twice, interleaved)
set -o pipefail
TAG=${1:-pcab}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    lib=$PWD/exp_libs/lib_$v.so; [ "$v" = cur ] && lib=$PWD/eth-consensus-specs_amd/libblsmi355x.so
    BLSMI355X_LIB=$lib timeout -k 10 120 python3 tools/percall_probe.py > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err \
      || { echo "$v FAILED"; tail -5 $OUT/$v.$rep.err; exit 1; }
    echo "$v $(cat $OUT/$v.$rep.json)"
  done
done | tee $OUT/summary.txt
