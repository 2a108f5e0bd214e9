#!/bin/bash
# Cost split of the scene-specialised kernel by duplicated sections (RT_EXP_DUP_*, via
# RTCORE_JIT_FLAGS): the time a second copy adds is that section's cost.
# usage: tools/dup_sweep.sh "CONFIGS"   (output lines: config flag ms/step kernel_ms)
set -e
mkdir -p gpurun_out
for cfg in $1; do
  for f in NONE RT_EXP_DUP_START RT_EXP_DUP_TRACE RT_EXP_DUP_SHADE; do
    flags=""; [ "$f" != NONE ] && flags="-D$f"
    RTCORE_JIT_FLAGS="$flags" timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/dup_${cfg}_$f.json 2> gpurun_out/dup_${cfg}_$f.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['kernel_ms'], d['config']['kernel_build'])" gpurun_out/dup_${cfg}_$f.json $cfg $f
  done
done
