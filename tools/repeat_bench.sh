#!/bin/bash
# Repeat a short bench under one jobs/queues/streams setting; stops at the first failure.
# Usage (via gpurun): bash tools/repeat_bench.sh TAG JOBS QUEUES SERIAL COUNT
set -o pipefail
TAG=$1; J=$2; Q=$3; S=$4; N=$5; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
envs="BLS_FAV_JOBS_INIT=$J GPU_MAX_HW_QUEUES=$Q"; [ "$S" = 1 ] && envs="$envs BLS_SERIAL=1"
for i in $(seq 1 $N); do
  env $envs timeout -k 10 120 python3 bench.py --steps 40 --warmup 3 --no-cpu --no-percall --no-e2e --roofline-passes 0 \
    > $OUT/r$i.json 2> $OUT/r$i.err || { echo "run $i FAILED rc=$?"; tail -2 $OUT/r$i.err | cut -c1-200; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/r$i.json')); print('run $i', d['value'])"
done
