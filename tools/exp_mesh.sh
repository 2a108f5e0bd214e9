#!/bin/bash
# A/B timing of library variants on the mesh config: tools/exp_mesh.sh base VARIANT...
# (a variant may repeat: each run's log is gpurun_out/<index>_<variant>_mesh1080.log)
steps=()
i=0
for v in "$@"; do
  i=$((i + 1))
  lib=""; [ "$v" != base ] && lib="RTCORE_LIB=raytracercore_amd/variants/$v/librtcore_hip.so"
  steps+=("$(printf %02d $i)_${v}_mesh1080|120|$lib python bench.py --no-cpu-baseline --config mesh1080 --steps 10 --warmup 3")
done
exec tools/gpu_steps.sh "${steps[@]}"
