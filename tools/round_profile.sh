#!/bin/bash
# One GPU-box session producing the round's evidence: GPU tests, smoke, bench
# lines for configs 3 (headline), 4/5 (8K), 6 (row f-1) and 8 (row f-4), rocprofv3
# kernel-trace summaries of the same commands, and the PMC passes for config 3.
# Every GPU step has its own limit; a crash/timeout/abort stops the script.
# SKIP_TESTS=1: no pytest/smoke; PROF_ONLY=1: no bench lines (rocprof steps only);
# BENCH_ONLY=1: stop before the rocprof steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r02_v1}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/status.txt"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  # (the per-dispatch traces stay on the box: gpurun merges back at most 64 MiB)
  rm -f "$OUT/$name"/run_kernel_trace.csv
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${PROF_ONLY:-0}" = 1 ] || step bench3 600 python bench.py
[ "${PROF_ONLY:-0}" = 1 ] || step bench3_short 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
[ "${PROF_ONLY:-0}" = 1 ] || step bench3_tg32 300 python bench.py --mode tile-gather --format rgba32f --no-cpu-baseline --no-host-output --tile-gather-steps 0
[ "${PROF_ONLY:-0}" = 1 ] || step bench3_tg8 300 python bench.py --mode tile-gather --format rgba8 --no-cpu-baseline --no-host-output --tile-gather-steps 0
[ "${PROF_ONLY:-0}" = 1 ] || step bench2 300 python bench.py --config 2 --no-alt --no-cpu-baseline
[ "${PROF_ONLY:-0}" = 1 ] || step bench4 300 python bench.py --config 4 --no-alt --no-cpu-baseline
[ "${PROF_ONLY:-0}" = 1 ] || step bench5 300 python bench.py --config 5 --no-alt --no-cpu-baseline
[ "${PROF_ONLY:-0}" = 1 ] || step bench6 300 python bench.py --config 6 --no-alt
[ "${PROF_ONLY:-0}" = 1 ] || step bench7 300 python bench.py --config 7 --no-alt --no-cpu-baseline
[ "${PROF_ONLY:-0}" = 1 ] || step bench8 300 python bench.py --config 8 --no-alt
[ "${PROF_ONLY:-0}" = 1 ] || step bench9 300 python bench.py --config 9 --no-alt
[ "${BENCH_ONLY:-0}" = 1 ] && { echo done; exit 0; }
step prof3 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 25 --warmup 3 --no-cpu-baseline --no-alt
RTM_LANES=1 step prof3_one_lane 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof3_one_lane" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 25 --warmup 3 --no-cpu-baseline --no-alt
step prof4 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof4" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 4 --steps 13 --warmup 2 --no-cpu-baseline --no-alt
step prof6 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof6" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 6 --steps 25 --warmup 3 --no-cpu-baseline --no-alt
step prof2 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof2" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt
step prof7 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof7" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 7 --steps 10 --warmup 2 --no-cpu-baseline --no-alt
step prof9 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof9" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 9 --steps 20 --warmup 5 --no-cpu-baseline --no-alt
step prof8 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof8" -o run --output-format csv -- python3 "$ROOT/bench.py" --config 8 --steps 13 --warmup 2 --no-cpu-baseline --no-alt
if [ "${PMC:-0}" = 1 ]; then
  TAG=$TAG CFG=3 BENCH_ARGS="--no-alt" step pmc3 1200 bash tools/profile_pmc.sh
fi
echo done
