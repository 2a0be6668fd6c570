#!/bin/bash
# [|x|] chains of cofactor clearing: wave program (BLS_XC_G=5) vs one lane per item (BLS_XC_G=1), 5 jobs.
set -o pipefail
for g in 5 1 5 1; do
  BLS_XC_G=$g bash tools/repeat_bench.sh xcab$g 5 20 0 1 || exit 1
done
