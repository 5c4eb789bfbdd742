#!/bin/bash
# Steps of 256 Mpixel worth: the driver's short invocation against the default run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02_v10s
mkdir -p $OUT
b() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['frames_per_step'], d['ms_per_step'], d['steps'], d['warmup'])" | tee -a $OUT/summary.txt
}
for r in 1 2; do
  b c3_default_$r --no-cpu-baseline --no-host-output --tile-gather-steps 0
  b c3_short_$r --steps 20 --warmup 5 --no-cpu-baseline --no-host-output --tile-gather-steps 0
  b c2_short_$r --config 2 --steps 20 --warmup 5 --no-cpu-baseline --no-host-output --tile-gather-steps 0 --no-alt
done
