#!/bin/bash
# GPU timeline of config 7 (512^2 ray-traced frames, 64 per launch): rocprofv3 kernel
# and memory-copy trace (per-dispatch start/end, queue) of a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r02_v8t}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-7}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace$CFG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-host-output --tile-gather-steps 0 > "$OUT/trace$CFG.log" 2>&1
rc=$?; tail -3 "$OUT/trace$CFG.log"; find "$OUT" -name "*.csv" | head; exit $rc
