#!/bin/bash
# A/B of environment settings (RTCORE_* switches, RTCORE_JIT_FLAGS) on bench configs, one bench
# run per (config, setting), kernel and step times printed side by side.
# usage: tools/ab_env.sh "CONFIGS" "VAR=VALUE ..." "VAR=VALUE ..." ...   ("-" = defaults)
set -e
mkdir -p gpurun_out
cfgs=$1; shift
for cfg in $cfgs; do
  k=0
  for setting in "$@"; do
    k=$((k+1))
    envs=""; [ "$setting" != "-" ] && envs="$setting"
    env $envs timeout -k 10 150 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_${cfg}_$k.json 2> gpurun_out/ab_${cfg}_$k.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], repr(sys.argv[3]), d['ms_per_step'], d['kernel_ms'], d['config']['kernel_build'])" gpurun_out/ab_${cfg}_$k.json $cfg "$setting"
  done
done
