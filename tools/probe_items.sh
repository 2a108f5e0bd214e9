#!/bin/bash
# item-length probe: per-ray rate vs item length and launch size (C2)
cd "${GRAFT_REPO_ROOT:-.}"
run() { name=$1; shift; echo "== $name"; env "$@" python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $SPPARG 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'])"; }
for rep in 1 2; do
SPPARG="" run c32_s256 RTCORE_X=1
SPPARG="" run c8_s256 RTCORE_PATH_CHUNKS=8
SPPARG="" run c16_s256 RTCORE_PATH_CHUNKS=16
SPPARG="--spp 1024" run c32_s1024 RTCORE_X=1
SPPARG="--spp 1024" run c128_s1024 RTCORE_PATH_CHUNKS=128
SPPARG="--spp 1024" run c64_s1024 RTCORE_PATH_CHUNKS=64
done
