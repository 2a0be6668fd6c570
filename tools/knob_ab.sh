#!/bin/bash
# A/B of env knobs at 5 jobs / 20 queues: each argument is VAR=VALUE (or "base"), one 40-step bench each.
set -o pipefail
i=0
for kv in "$@"; do
  i=$((i+1))
  if [ "$kv" = base ]; then envs=""; else envs="$kv"; fi
  env $envs bash tools/repeat_bench.sh knob$i 5 20 0 1 | sed "s/^/$kv /" || exit 1
done
