#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/status.txt"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline
fi
echo done
