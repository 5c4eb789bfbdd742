#!/bin/bash
# Builds librtm with a fixed bounds bug restored, into build/revert/ (outside the
# package: never loaded by the product), to show the bounds tests catch it.  Run on the GPU box: the named tests
# pass against librtm.so and must FAIL, with a nonzero rtm_ctx_oob_reads count, against
# the demo build.
#   tools/bounds_demo.sh            -> librtm_noguard.so  (-DRTM_TEST_REVERT_MASK_GUARD:
#       the round-3 RT mask over-read)
#       RTM_LIB=$PWD/build/revert/librtm_noguard.so python -m pytest tests/test_bounds.py
#   tools/bounds_demo.sh slots      -> librtm_allslots.so (-DRTM_TEST_REVERT_SLOT_MASKS: the
#       pre-dfafeba primitive masks with every slot bit set, round-4 fault study)
#       RTM_LIB=$PWD/build/revert/librtm_allslots.so python -m pytest tests/test_id_bounds.py
#   tools/bounds_demo.sh union      -> librtm_emptyunion.so (-DRTM_TEST_REVERT_EMPTY_UNION: the
#       round-3 empty sphere union that met the top-left strip)
#       RTM_LIB=$PWD/build/revert/librtm_emptyunion.so python -m pytest tests/test_stale_state_fuzz.py
set -euo pipefail
case "${1:-guard}" in
  guard) DEF=-DRTM_TEST_REVERT_MASK_GUARD; OUT=librtm_noguard.so ;;
  slots) DEF=-DRTM_TEST_REVERT_SLOT_MASKS; OUT=librtm_allslots.so ;;
  union) DEF=-DRTM_TEST_REVERT_EMPTY_UNION; OUT=librtm_emptyunion.so ;;
  *) echo "usage: $0 [guard|slots|union]" >&2; exit 2 ;;
esac
cd "$(dirname "$0")/../2018rustraytracer_amd/csrc"
make -s  # the other objects
B=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
    --offload-arch=gfx950 $DEF -c rtm_kernels.hip -o "$B/rtm_kernels.o"
D=../../build/revert
mkdir -p "$D"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$D/$OUT" "$B/rtm_kernels.o" rtm_encode.o \
    rtm_api.o rtm_group.o -ldl
rm -rf "$B"
echo "built $(cd "$D" && pwd)/$OUT"
