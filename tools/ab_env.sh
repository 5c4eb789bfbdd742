#!/bin/bash
# A/B of library environment switches on bench.py lines, interleaved rounds in one
# GPU session.  Usage: bash tools/ab_env.sh OUTDIR "CONFIGS" "VARIANT1;VARIANT2;..." [ROUNDS] [extra bench args]
# A variant is a space-separated list of VAR=value (or "-" for the defaults).
set -o pipefail
export TMPDIR=/tmp
O=$1; CFGS=$2; VARS=$3; ROUNDS=${4:-2}; shift 4; EXTRA="$*"
mkdir -p "$O"
IFS=';' read -ra VA <<< "$VARS"
for c in $CFGS; do for r in $(seq 1 "$ROUNDS"); do for vi in "${!VA[@]}"; do
  v=${VA[$vi]}
  f="$O/b${c}_v${vi}_r$r.log"
  if [ "$v" = "-" ]; then envs=(); else read -ra envs <<< "$v"; fi
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --config "$c" --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output $EXTRA > "$f" 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 "$f"; exit $rc; }
  python - "$f" "$c" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(f"config {sys.argv[2]} [{sys.argv[3]}] {d['value']:.0f} Mpix/s, {d['ms_per_frame']*1e3:.2f} us/frame, "
      f"kernels {d['kernels']}, one-lane {(d.get('one_lane') or {}).get('value')}", flush=True)
PY
done; done; done
