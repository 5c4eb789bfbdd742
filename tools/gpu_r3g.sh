#!/bin/bash
# Frames-per-launch cliff at 3840x2160 (RTM_BATCH=8 ran at 150 vs 251 Gpix/s):
# rocprofv3 kernel stats at B = 4 and 8, lanes as run and one lane.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r02_v8c
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "4 2" "8 2" "8 1" "4 1"; do
  set -- $v
  timeout -k 10 200 env RTM_BATCH=$1 RTM_LANES=$2 rocprofv3 --kernel-trace --stats -d "$OUT/b$1_l$2" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output > "$OUT/b$1_l$2.log" 2>&1
  rc=$?; echo "b$1 l$2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b$1_l$2.log') if l.startswith('{')][-1]); print(d['value'], d['lanes'], d['frames_per_launch'], d['kernels'])"
  cut -d, -f1-4 "$OUT/b$1_l$2/run_kernel_stats.csv" | head -4
done
