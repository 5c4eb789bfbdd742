#!/bin/bash
# Builds an A/B variant of librtm: rtm_kernels.hip with extra compile flags (e.g. a
# -DRTM_AB_* switch under test), linked with the tree's other objects, as
# 2018rustraytracer_amd/librtm_NAME.so.  Load it with RTM_LIB=<path> (tools/ab_env.sh).
# The product build (make) never defines an RTM_AB_* switch.
#   bash tools/ab_lib.sh NAME "FLAGS" ["API_FLAGS"]   (API_FLAGS: rtm_api.cpp rebuilt with them)
set -euo pipefail
NAME=$1; FLAGS=${2:-}; API_FLAGS=${3:-}
cd "$(dirname "$0")/../2018rustraytracer_amd/csrc"
make -s  # the other objects
B=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
    --offload-arch=gfx950 $FLAGS -c rtm_kernels.hip -o "$B/rtm_kernels.o"
API=rtm_api.o
if [ -n "$API_FLAGS" ]; then
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
      $API_FLAGS -c rtm_api.cpp -o "$B/rtm_api.o"
  API="$B/rtm_api.o"
fi
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "../librtm_$NAME.so" "$B/rtm_kernels.o" rtm_encode.o \
    "$API" rtm_group.o -ldl
rm -rf "$B"
echo "built $(cd .. && pwd)/librtm_$NAME.so"
