#!/bin/bash
# Host-phase profile (RTM_HOST_PROF=1) of frame sequences: config 7 (512^2 ray-traced,
# host-bound), config 2 and config 3, through the enqueue probe and bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02_v8h}
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
export RTM_HOST_PROF=1
CFG=7 N=1024 step enq7 120 python tools/probes/host_enqueue.py
CFG=7 N=64 step enq7_64 120 python tools/probes/host_enqueue.py
CFG=2 N=512 step enq2 120 python tools/probes/host_enqueue.py
CFG=3 N=256 step enq3 120 python tools/probes/host_enqueue.py
step bench7 300 python bench.py --config 7 --no-alt --no-cpu-baseline --no-host-output --tile-gather-steps 0
step bench2 300 python bench.py --config 2 --no-alt --no-cpu-baseline --no-host-output --tile-gather-steps 0
echo done
