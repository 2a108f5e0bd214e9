#!/bin/bash
# C4 refill / leaf-step thresholds (RTCORE_BVH_REFILL, RTCORE_BVH_SPEC), two alternating rounds
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for cfg in "28 12" "24 12" "20 12" "32 12" "28 16" "24 10"; do
    set -- $cfg
    line=$(RTCORE_BVH_REFILL=$1 RTCORE_BVH_SPEC=$2 timeout -k 10 120 python3 bench.py --no-cpu-baseline --config mesh1080 --steps 10 --warmup 3 2>/dev/null | tail -1) || exit 1
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', 'refill $1 spec $2', d['kernel_ms'], d['ms_per_step'])"
  done
done
