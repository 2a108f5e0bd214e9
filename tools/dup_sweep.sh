#!/bin/bash
# Cost split of the path kernel by duplicated or removed sections (tools/exp_patch.py variants:
# build them on the CPU first, e.g. `for v in NO_TRACE DUP_SHADE DUP_START; do python
# tools/exp_patch.py $v $v; done`): the time a second copy adds is that section's cost.
# usage: tools/dup_sweep.sh "CONFIGS" "VARIANTS"   (output lines: config variant ms/step kernel_ms)
set -e
mkdir -p gpurun_out
for cfg in $1; do
  for v in base $2; do
    lib=""; [ "$v" != base ] && lib="raytracercore_amd/variants/$v/librtcore_hip.so"
    RTCORE_LIB="$lib" timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/dup_${cfg}_$v.json 2> gpurun_out/dup_${cfg}_$v.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['kernel_ms'], d['config']['kernel_build'])" gpurun_out/dup_${cfg}_$v.json $cfg $v
  done
done
