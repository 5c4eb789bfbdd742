#!/bin/bash
# Session check after a library change: GPU tests, smoke, the default bench line,
# rocprofv3 kernel traces (lanes as run, and one lane) and the config-3 PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r02_v4}
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
step bench3 600 python bench.py ${BENCH_ARGS:-}
step prof3 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 25 --warmup 3 --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output
RTM_LANES=1 step prof3_one_lane 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof3_one_lane" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 25 --warmup 3 --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output
if [ "${PMC:-1}" = 1 ]; then
  TAG=$TAG CFG=${CFG:-3} BENCH_ARGS="--no-alt" step pmc3 1200 bash tools/profile_pmc.sh
fi
echo done
