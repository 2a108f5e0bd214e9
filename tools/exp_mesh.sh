#!/bin/bash
# A/B timing of library variants on the mesh config: tools/exp_mesh.sh base VARIANT...
steps=()
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib="RTCORE_LIB=raytracercore_amd/variants/$v/librtcore_hip.so"
  steps+=("${v}_mesh1080|120|$lib python bench.py --no-cpu-baseline --config mesh1080")
done
exec tools/gpu_steps.sh "${steps[@]}"
