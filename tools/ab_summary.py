#!/usr/bin/env python3
"""One line per bench log of an A/B directory (tools/ab_env.sh): value,
us/frame, kernel durations, one-lane value."""
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "*.log"))):
        lines = [l for l in open(f) if l.startswith("{")]
        if not lines:
            continue
        r = json.loads(lines[0])
        print(f"{os.path.basename(f)}: config {r['config']['config_id']} {r['value']:.0f} Mpix/s, "
              f"{r.get('ms_per_frame', r['ms_per_step']) * 1e3:.2f} us/frame, kernels {r['kernels']}, "
              f"lanes {r.get('lanes')}, one-lane {(r.get('one_lane') or {}).get('value')}")
