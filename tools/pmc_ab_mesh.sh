#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
P="python3 bench.py --no-cpu-baseline --config mesh1080 --steps 3 --warmup 1"
for v in base old; do
  lib=""; [ "$v" != base ] && lib="raytracercore_amd/variants/$v/librtcore_hip.so"
  out=gpurun_out/pmc_rng/$v; mkdir -p $out
  RTCORE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o pmc -- $P > $out/p1.log 2>&1 || { echo "$v p1 failed"; exit 1; }
  RTCORE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/p2 -o pmc -- $P > $out/p2.log 2>&1 || { echo "$v p2 failed"; exit 1; }
  echo "$v done"
done
