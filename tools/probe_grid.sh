#!/bin/bash
# Probe: blocks per CU of the scene-specialised launch (RTCORE_GRID_BPC) on small and large launches.
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for bpc in 8 6 4 3 2; do
    for c in bounce256 bounce1080; do
      line=$(RTCORE_GRID_BPC=$bpc timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 1
      echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', 'bpc$bpc', '$c', d['kernel_ms'], d['ms_per_step'], d['value'])"
    done
  done
done
