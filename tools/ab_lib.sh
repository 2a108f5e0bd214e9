#!/bin/bash
# Same-call A/B of library variants on the headline configs: tools/ab_lib.sh "CONFIGS" base|VARIANT ...
# (VARIANT = raytracercore_amd/variants/VARIANT, tools/build_variant.sh); two alternating rounds,
# one bench line per variant and config (kernel ms and value).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cfgs=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="raytracercore_amd/variants/$v/librtcore_hip.so"
    for c in $cfgs; do
      line=$(RTCORE_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $c --steps 10 --warmup 3 2>/dev/null | tail -1)
      rc=$?
      [ $rc -ne 0 ] && { echo "$v $c rc=$rc"; exit $rc; }
      echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep', '$v', '$c', d['value'], d['ms_per_step'], d['kernel_ms'])"
    done
  done
done
