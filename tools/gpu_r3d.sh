#!/bin/bash
# Config 7 (512^2, host/queue-bound) env sweep through bench.py: hardware queues,
# upload stream, lanes, frames per launch; 2 interleaved rounds.  CFG env: config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02_v8q}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-7}
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config $CFG --no-alt --no-cpu-baseline --no-host-output --tile-gather-steps 0 --steps 120 --warmup 20 > "$OUT/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$OUT/$name.log"; exit $rc; }
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['lanes'], d['frames_per_launch'], (d.get('alt_fused_shadow') or {}).get('value'))" | tee -a "$OUT/summary.txt"
}
for r in 1 2; do
  for c in ${CFGS:-7}; do
    CFG=$c
    for v in ${VARIANTS:-X=1}; do
      run c${c}_${v//[=,]/_}_$r $v
    done
  done
done
echo done
