#!/bin/bash
# C4 (mesh 1080p x 64 spp) under wide-collapse variants: "name|ENV=... ENV=..." per argument;
# one bench run each (kernel ms, node visits and primitive tests per ray segment in the JSON line).
steps=()
for spec in "$@"; do
  name="${spec%%|*}"; envs="${spec#*|}"
  steps+=("wide_${name}|150|env $envs python bench.py --no-cpu-baseline --config mesh1080 --steps 5 --warmup 1")
done
exec tools/gpu_steps.sh "${steps[@]}"
