#!/bin/bash
# Re-entry check (fresh container, rebuilt .so): GPU tests, smoke, the default bench
# line, and the host-enqueue probe for the small ray-traced frames (config 7) next to
# config 3, to see how much of config 7's frame time is host work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r02_v8}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 137 ] || [ "$rc" -gt 128 ]; }
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/status.txt"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench3 600 python bench.py
CFG=7 N=64 step enq7_64 120 python tools/probes/host_enqueue.py
CFG=7 N=1024 step enq7_1024 120 python tools/probes/host_enqueue.py
CFG=3 N=64 step enq3_64 120 python tools/probes/host_enqueue.py
step bench7 300 python bench.py --config 7 --no-alt --no-cpu-baseline --no-host-output --tile-gather-steps 0
echo done
