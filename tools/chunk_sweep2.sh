#!/bin/bash
# chunks per pixel (RTCORE_PATH_CHUNKS) on C2 and C5 after the round-6 stream change; two rounds
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for cfg in "bounce1080 0" "bounce1080 24" "bounce1080 48" "die4k 0" "die4k 4" "die4k 16"; do
    set -- $cfg
    env=""; [ "$2" != 0 ] && env="RTCORE_PATH_CHUNKS=$2"
    line=$(env $env timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $1 --steps 10 --warmup 3 2>/dev/null | tail -1) || exit 1
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', '$1', 'chunks $2', d['kernel_ms'], d['ms_per_step'])"
  done
done
