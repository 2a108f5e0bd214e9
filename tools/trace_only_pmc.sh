#!/bin/bash
# PMC passes over the trace-only kernel fed in the megakernel's order and in a globally sorted
# (ray-binned) order, 8 waves per SIMD.  Dispatch order per process: for each
# order, the instrumented launch then the timed one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp TRACE_ORDERS=pixel_then_bounce,octant_then_origin TRACE_WAVES=8
out=gpurun_out/trace_pmc
mkdir -p $out
set -e
timeout -k 10 150 rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $out/pmct -o pmc -- python3 tools/trace_only.py 4 > $out/pmct.log 2>&1
timeout -k 10 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $out/pmcl2 -o pmc -- python3 tools/trace_only.py 4 > $out/pmcl2.log 2>&1
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/pmcv -o pmc -- python3 tools/trace_only.py 4 > $out/pmcv.log 2>&1
echo done
