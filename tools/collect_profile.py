#!/usr/bin/env python3
"""Copy a round-profile run (tools/round_profile.sh: gpurun_out/<TAG>/) into
profiles/: each bench log's JSON line as <TAG>_bench_<name>.json, each rocprofv3
kernel-stats CSV as <TAG>_kernel_stats_<name>.csv, the GPU-test and smoke logs."""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", tag)
dst = os.path.join(ROOT, "profiles")
for f in sorted(glob.glob(os.path.join(src, "bench*.log"))):
    lines = [l for l in open(f) if l.startswith("{")]
    if lines:
        name = os.path.basename(f)[len("bench"):-len(".log")]
        name = "config" + name if name[:1].isdigit() else name
        with open(os.path.join(dst, f"{tag}_bench_{name}.json"), "w") as o:
            json.dump(json.loads(lines[0]), o, indent=1)
for f in sorted(glob.glob(os.path.join(src, "prof*", "run_kernel_stats.csv"))):
    name = os.path.basename(os.path.dirname(f))[len("prof"):]
    name = "config" + name if name[:1].isdigit() else name
    shutil.copy(f, os.path.join(dst, f"{tag}_kernel_stats_{name}.csv"))
for n in ("pytest_gpu", "smoke", "status"):
    for ext in (".log", ".txt"):
        f = os.path.join(src, n + ext)
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, f"{tag}_{n}{ext}"))
print(sorted(os.path.basename(p) for p in glob.glob(os.path.join(dst, tag + "_*"))))
