#!/bin/bash
# New auto frames-per-launch rule (64 Mpixel worth, batch tables pulled): GPU tests,
# then per-config A/B against the old batch sizes and one size up, and the
# tile-gather lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02_v10b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFGS="3" VARIANTS="X=1 RTM_BATCH=4 RTM_BATCH=16" TAG=r02_v10b bash tools/gpu_r3d.sh || exit 1
CFGS="2" VARIANTS="X=1 RTM_BATCH=4 RTM_BATCH=32" TAG=r02_v10b bash tools/gpu_r3d.sh || exit 1
CFGS="4 5" VARIANTS="X=1 RTM_BATCH=4" TAG=r02_v10b bash tools/gpu_r3d.sh || exit 1
CFGS="6 8 9" VARIANTS="X=1 RTM_BATCH=4" TAG=r02_v10b bash tools/gpu_r3d.sh || exit 1
for f in rgba32f rgba8; do
  timeout -k 10 300 python bench.py --mode tile-gather --format $f --no-cpu-baseline --no-host-output --tile-gather-steps 0 > $OUT/tg_$f.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$OUT/tg_$f.log') if l.startswith('{')][-1]); print('tg $f', d['value'], d['frames_per_launch'])"
done
