#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
for v in base w8; do
  lib=""; [ "$v" != base ] && lib="raytracercore_amd/variants/$v/librtcore_hip.so"
  for hot in 64 0; do
    line=$(RTCORE_HOT_NODES=$hot RTCORE_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --config mesh1080 --steps 10 --warmup 3 2>/dev/null | tail -1) || exit 1
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', '$v', 'hot$hot', d['kernel_ms'], d['ms_per_step'])"
  done
done
done
