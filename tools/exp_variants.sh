#!/bin/bash
# A/B timing of library variants on the brute-force configs: tools/exp_variants.sh base VARIANT...
steps=()
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib="RTCORE_LIB=raytracercore_amd/variants/$v/librtcore_hip.so"
  for c in bounce1080 die1080; do
    steps+=("${v}_$c|90|$lib python bench.py --no-cpu-baseline --config $c")
  done
done
exec tools/gpu_steps.sh "${steps[@]}"
