#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box via tools/gpu_steps.sh):
#   trace: --kernel-trace --stats with the driver's step counts (20 timed + 5 warm-up), so the
#          kernel-trace average is the steady state bench.py's kernel_ms reports;
#   pmc1..pmc7: counter passes (5 steps), each its own run, no tracing domains with --pmc.
# usage: tools/profile.sh TAG [bench args...]
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
set -e
rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > "$out/trace.log" 2>&1
P="python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 $*"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d "$out/pmc1" -o pmc -- $P > "$out/pmc1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc2" -o pmc -- $P > "$out/pmc2.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc3" -o pmc -- $P > "$out/pmc3.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VALU_CVT --output-format csv -d "$out/pmc4" -o pmc -- $P > "$out/pmc4.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_LDS_BANK_CONFLICT --output-format csv -d "$out/pmc5" -o pmc -- $P > "$out/pmc5.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum --output-format csv -d "$out/pmc6" -o pmc -- $P > "$out/pmc6.log" 2>&1
# the vector-memory pipeline: texture addresser, L1 tag lookups, L1 -> L2 requests
timeout -s KILL 150 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d "$out/pmc7" -o pmc -- $P > "$out/pmc7.log" 2>&1
echo "profile $tag done"
