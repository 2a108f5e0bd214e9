#!/bin/bash
# One GPU call that refreshes a round's evidence: rocprofv3 trace + PMC passes of the three
# profiled configs (tools/profile.sh) and the bench lines of every config with the CPU baseline.
# usage (on the GPU box): tools/round_profiles.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tools/gpu_steps.sh \
  "prof_c2|420|tools/profile.sh bounce1080" \
  "prof_c3|420|tools/profile.sh die1080 --config die1080" \
  "prof_c4|600|tools/profile.sh mesh1080 --config mesh1080" \
  "bench_bounce1080|240|python3 bench.py --steps 20 --warmup 5" \
  "bench_die1080|240|python3 bench.py --config die1080 --steps 20 --warmup 5" \
  "bench_mesh1080|300|python3 bench.py --config mesh1080 --steps 20 --warmup 5" \
  "bench_die4k|300|python3 bench.py --config die4k --steps 10 --warmup 3" \
  "bench_bounce256|120|python3 bench.py --config bounce256 --steps 20 --warmup 5"
exit $?
