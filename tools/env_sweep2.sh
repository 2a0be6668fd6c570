#!/bin/bash
# Throughput vs FAV jobs in flight, streams per job (BLS_SERIAL=1: one) and hardware queues.
# Usage (via gpurun): bash tools/env_sweep2.sh TAG "JOBS:QUEUES:SERIAL ..."
set -o pipefail
TAG=${1:-sweep}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in $2; do
  IFS=: read -r J Q S <<< "$cfg"
  envs="BLS_FAV_JOBS_INIT=$J GPU_MAX_HW_QUEUES=$Q"
  [ "$S" = 1 ] && envs="$envs BLS_SERIAL=1"
  env $envs timeout -k 10 150 python3 bench.py --steps 30 --warmup 3 --no-cpu --no-percall --no-e2e --roofline-passes 0 \
    > $OUT/b_${J}_${Q}_${S}.json 2> $OUT/b_${J}_${Q}_${S}.err
  rc=$?
  echo "$cfg rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/b_${J}_${Q}_${S}.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -3 $OUT/b_${J}_${Q}_${S}.err; [ $rc -ge 124 ] && exit 1; fi
done
