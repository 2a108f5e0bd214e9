#!/bin/bash
# items per dispenser atomic (RTCORE_POOL_MUL x 64) with the 24-chunk items, C2 and C3, two rounds
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for cfg in "bounce1080 0" "bounce1080 2" "die1080 0" "die1080 2" "die1080 8"; do
    set -- $cfg
    env=""; [ "$2" != 0 ] && env="RTCORE_POOL_MUL=$2"
    line=$(env $env timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $1 --steps 10 --warmup 3 2>/dev/null | tail -1) || exit 1
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', '$1', 'pool_mul $2', d['kernel_ms'], d['ms_per_step'])"
  done
done
