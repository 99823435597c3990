#!/usr/bin/env bash
# Build a library variant for A/B runs: tools/build_variant.sh <name> "<-D defines>"
# -> rvgrt_amd/variants/<name>/librvgrt_hip.so (selected at run time with RVGRT_LIB).
set -e
cd "$(dirname "$0")/.."
make -s -C rvgrt_amd/csrc OUT=../variants/$1/librvgrt_hip.so OBJDIR=build_$1 DEFS="$2" -j3 2>&1 | grep -v "hip-link" || true
test -f rvgrt_amd/variants/$1/librvgrt_hip.so
