#!/bin/bash
# Builds librtm with the round-3 RT mask over-read restored (-DRTM_TEST_REVERT_MASK_GUARD)
# as 2018rustraytracer_amd/librtm_noguard.so (never loaded by the product).  Run on the
# GPU box: tests/test_bounds.py passes against librtm.so and must FAIL, with a nonzero
# rtm_ctx_oob_reads count, against this build:
#   RTM_LIB=$PWD/2018rustraytracer_amd/librtm_noguard.so python -m pytest tests/test_bounds.py
set -euo pipefail
cd "$(dirname "$0")/../2018rustraytracer_amd/csrc"
make -s  # the other objects
B=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
    --offload-arch=gfx950 -DRTM_TEST_REVERT_MASK_GUARD -c rtm_kernels.hip -o "$B/rtm_kernels.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../librtm_noguard.so "$B/rtm_kernels.o" rtm_encode.o \
    rtm_api.o rtm_group.o -ldl
rm -rf "$B"
echo "built $(cd .. && pwd)/librtm_noguard.so"
