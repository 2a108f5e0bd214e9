#!/bin/bash
# Build an experimental variant of the library: tools/build_variant.sh NAME "-DFLAG=..."
# -> raytracercore_amd/variants/NAME/librtcore_hip.so (load with RTCORE_LIB=<that path>)
set -e
cd "$(dirname "$0")/../raytracercore_amd/csrc"
mkdir -p ../variants/$1
make -s OBJ=_obj_$1 OUT=../variants/$1 EXTRA="$2" 2>&1 | grep -E "error" || true
ls -la ../variants/$1/librtcore_hip.so
