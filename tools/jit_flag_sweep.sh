#!/bin/bash
# A/B of compile flags of the scene-specialised kernel (RTCORE_JIT_FLAGS) on one bench config.
# usage: tools/jit_flag_sweep.sh CONFIG "FLAGS A" "FLAGS B" ...   ("-" = no extra flags)
set -e
mkdir -p gpurun_out
cfg=$1; shift
k=0
for f in "$@"; do
  k=$((k+1))
  flags="$f"; [ "$f" = "-" ] && flags=""
  RTCORE_JIT_FLAGS="$flags" timeout -k 10 150 python bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline \
    > gpurun_out/jf_${cfg}_$k.json 2> gpurun_out/jf_${cfg}_$k.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], repr(sys.argv[3]), d['ms_per_step'], d['kernel_ms'])" gpurun_out/jf_${cfg}_$k.json $cfg "$f"
done
