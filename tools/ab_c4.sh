#!/bin/bash
# C4 A/B of library variants with their counters (run on the GPU box through tools/gpu_steps.sh):
# per variant one timed bench run and three PMC passes (writes; L1 / L2 requests and the texture
# addresser; L2 hits), each pass its own rocprofv3 run.
# usage: tools/ab_c4.sh TAG base|VARIANT ...   (VARIANT = raytracercore_amd/variants/VARIANT)
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
steps=()
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib="RTCORE_LIB=raytracercore_amd/variants/$v/librtcore_hip.so"
  out=gpurun_out/ab_${tag}/$v
  P="python3 bench.py --no-cpu-baseline --config mesh1080 --steps 3 --warmup 1"
  steps+=("${tag}_${v}_time|150|mkdir -p $out && $lib python3 bench.py --no-cpu-baseline --config mesh1080 --steps 10 --warmup 3 > $out/bench.json")
  steps+=("${tag}_${v}_pmcw|90|$lib rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmcw -o pmc -- $P")
  steps+=("${tag}_${v}_pmct|90|$lib rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $out/pmct -o pmc -- $P")
  steps+=("${tag}_${v}_pmcl2|90|$lib rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $out/pmcl2 -o pmc -- $P")
done
exec tools/gpu_steps.sh "${steps[@]}"
