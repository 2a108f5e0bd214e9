#!/bin/bash
# Same-call A/B of scene-specialised build flags on C2 and C3: tools/ab_jit.sh TAG "FLAGS_A" "FLAGS_B" ...
# ("" = the default build); each config and flag set twice, alternating.
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
steps=()
for rep in 1 2; do
  i=0
  for f in "$@"; do
    for cfg in bounce1080 die1080; do
      steps+=("${tag}_${cfg}_${i}_${rep}|150|RTCORE_JIT_FLAGS='$f' python3 bench.py --no-cpu-baseline --config $cfg --steps 10 --warmup 3")
    done
    i=$((i+1))
  done
done
exec tools/gpu_steps.sh "${steps[@]}"
