#!/bin/bash
# C2 / C3 rates against the number of job slots and hardware queues (one bench run per setting).
# Usage (via gpurun): bash tools/jobs_sweep.sh TAG "JOBS:QUEUES" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for jq in "$@"; do
  j=${jq%%:*}; q=${jq##*:}
  BLS_FAV_JOBS_INIT=$j GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu --no-percall --no-e2e --c4-steps 0 --c5-steps 0 --no-regload \
    --no-parity > $OUT/j${j}_q${q}.json 2> $OUT/j${j}_q${q}.err || { echo "$jq FAILED"; tail -3 $OUT/j${j}_q${q}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/j${j}_q${q}.json')); print('jobs $j queues $q', d['value'], d['c3']['fav_s'], d['c3']['ms_per_epoch'])"
done
