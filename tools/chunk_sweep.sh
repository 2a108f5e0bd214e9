#!/bin/bash
# Work-item length sweep: RTCORE_PATH_CHUNKS (chunks per pixel) against kernel time per config.
# usage: tools/chunk_sweep.sh "CONFIGS" "CHUNKS"   (output: gpurun_out/chunks_<cfg>_<n>.json)
set -e
mkdir -p gpurun_out
for cfg in $1; do
  for n in $2; do
    RTCORE_PATH_CHUNKS=$n timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/chunks_${cfg}_${n}.json 2> gpurun_out/chunks_${cfg}_${n}.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['value']/1e3,1))" gpurun_out/chunks_${cfg}_${n}.json $cfg $n
  done
done
