#!/bin/bash
# chunks per pixel (RTCORE_PATH_CHUNKS) on C2 and C3: 16 / 20 / 24 / 28 / default 32, two rounds
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for c in bounce1080 die1080; do
    for k in 0 16 20 24 28; do
      env=""; [ "$k" != 0 ] && env="RTCORE_PATH_CHUNKS=$k"
      line=$(env $env timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $c --steps 10 --warmup 3 2>/dev/null | tail -1) || exit 1
      echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', '$c', 'chunks $k', d['kernel_ms'], d['ms_per_step'])"
    done
  done
done
