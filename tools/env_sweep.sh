#!/bin/bash
# A/B sweep of the C2 bench line over environment settings.
# Usage (via gpurun): bash tools/env_sweep.sh TAG "NAME=V[,NAME2=V2] ..."
set -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for cfg in $2; do
  tag=${cfg//[=,]/_}
  env ${cfg//,/ } timeout -k 10 240 python -u bench.py --steps 40 --warmup 2 --no-cpu --no-e2e \
    > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
  python3 -c "import json,sys; j=json.load(open(sys.argv[1])); print(sys.argv[2], round(j['value']), 'FAV/s', j['ms_per_step'], 'ms', {k: v for k, v in j['kernels_avg_ms'].items() if 'miller' in k})" "$OUT/bench_$tag.json" "$cfg"
done
