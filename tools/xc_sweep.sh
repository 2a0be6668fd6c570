#!/bin/bash
# Throughput vs items per workgroup of the [|x|] chain wave program (BLS_XC_G).
set -o pipefail
for g in 4 5 6; do
  BLS_XC_G=$g bash tools/repeat_bench.sh xc$g 5 20 0 2 || exit 1
done
