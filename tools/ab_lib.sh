#!/bin/bash
# Builds an A/B variant of librtm: rtm_kernels.hip with a patch applied (PATCH: a unified
# diff against the tree, e.g. the variant's constants or kernel body) and/or extra compile
# flags, linked with the tree's other objects, as build/ab/librtm_NAME.so (outside the
# package).  Load it with RTM_LIB=<path> (tools/ab_env.sh).  The product source holds no
# A/B switch: a variant lives only in its patch.
#   PATCH=variant.diff bash tools/ab_lib.sh NAME ["FLAGS"] ["API_FLAGS"]   (API_FLAGS: rtm_api.cpp rebuilt with them)
set -euo pipefail
NAME=$1; FLAGS=${2:-}; API_FLAGS=${3:-}
if [ -n "${PATCH:-}" ]; then PATCH=$(realpath "$PATCH"); fi
cd "$(dirname "$0")/../2018rustraytracer_amd/csrc"
make -s  # the other objects
B=$(mktemp -d)
cp rtm_kernels.hip rtm_kernels.h rtm_api.cpp rtm_internal.h rtm_encode.h "$B/"
if [ -n "${PATCH:-}" ]; then (cd "$B" && patch -s -p3 < "$PATCH"); fi
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
    -I"$PWD" --offload-arch=gfx950 $FLAGS -c "$B/rtm_kernels.hip" -o "$B/rtm_kernels.o"
API=rtm_api.o
if [ -n "$API_FLAGS" ] || { [ -n "${PATCH:-}" ] && grep -q "rtm_api.cpp" "$PATCH"; }; then
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
      -I"$PWD" $API_FLAGS -c "$B/rtm_api.cpp" -o "$B/rtm_api.o"
  API="$B/rtm_api.o"
fi
D=../../build/ab
mkdir -p "$D"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$D/librtm_$NAME.so" "$B/rtm_kernels.o" rtm_encode.o \
    "$API" rtm_group.o -ldl
rm -rf "$B"
echo "built $(cd "$D" && pwd)/librtm_$NAME.so"
