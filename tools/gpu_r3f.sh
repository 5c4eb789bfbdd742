#!/bin/bash
# After the shared-table upload and the prebuilt swap-chain pointer array: the batch
# tests, then bench lines for configs 7, 2, 3 with the host-phase profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02_v8f}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/status.txt"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  tail -2 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "step failed, stopping"; exit $rc; }
}
step tests 300 python -u -m pytest tests/test_raytrace.py tests/test_sdf.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for c in 7 2 3; do
  RTM_HOST_PROF=1 step bench$c 300 python bench.py --config $c --no-cpu-baseline --no-host-output --tile-gather-steps 0
done
echo done
