#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes into per-kernel averages per dispatch.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads (x2 applied, flagged), WRITE_SIZE is exact for
16-B-per-lane streaming stores.  The counters include Infinity-Cache hits."""
import argparse
import csv
import glob
import hashlib
import json
import os
import re
import time
from collections import defaultdict


def short(name):
    m = re.search(r"(shadow_\w+_kernel|eye_\w+_kernel|frame_pipe_kernel|rt_\w+_kernel|upload_kernel|"
                  r"vp_\w+_kernel|fill_kernel|encode_rgb8_kernel|ppm_\w+_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            did = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per[(k, did)][row["Counter_Name"]] += float(row["Counter_Value"])
        for (k, did), cs in per.items():
            for c, v in cs.items():
                vals[k][c].append(v)
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            durs[short(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    # frames per launch of the bench run the passes profiled (rtm_ctx_set_batch): the
    # per-dispatch bytes cover that many frames
    fpl = 1
    for f in sorted(glob.glob(os.path.join(a.dir, "*.log"))):
        for line in open(f, errors="replace"):
            if line.startswith("{"):
                try:
                    fpl = int(json.loads(line).get("frames_per_launch") or 1)
                except ValueError:
                    pass
                break
    # the librtm.so the passes profiled (bench.py cites a summary only for the same build)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "2018rustraytracer_amd", "librtm.so"), "rb") as f:
        build_id = hashlib.sha256(f.read()).hexdigest()[:16]
    out = {"config": a.config, "tag": a.tag, "source": "rocprofv3 --pmc, one pass per counter group",
           "librtm_build_id": build_id, "generated_unix": int(time.time()),
           "frames_per_launch": fpl, "kernels": {}}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if durs.get(k):
            d["avg_duration_ns_profiled"] = sum(durs[k]) / len(durs[k])
        if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
            fetch = d.get("FETCH_SIZE", 0.0) * 1024 * 2  # gfx950: FETCH_SIZE reads 1/2 of wide streaming reads
            write = d.get("WRITE_SIZE", 0.0) * 1024
            d["hbm_bytes_per_launch"] = int(fetch + write)
            d["hbm_bytes_note"] = "(FETCH_SIZE*2 + WRITE_SIZE) KiB->B; includes Infinity-Cache hits"
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
            d["salu_insts_per_wave"] = d.get("SQ_INSTS_SALU", 0) / d["SQ_WAVES"]
        timed_shadow = k.startswith("shadow_") and not k.startswith("shadow_pass_kernel<true")  # (<true>: stats)
        name = ("shadow_pass" if timed_shadow else
                "eye_pass" if k.startswith(("eye_pass_kernel<false, false", "eye_batch_kernel<false",
                                             "eye_sdf_kernel", "eye_sdf_batch_kernel", "eye_pass8_kernel",
                                             "eye_batch8_kernel")) else
                "eye_pass_fused" if k.startswith(("eye_pass_kernel<true, false", "eye_batch_kernel<true")) else k)
        if name in out["kernels"] and out["kernels"][name]["dispatches"] >= d["dispatches"]:
            out["kernels"][k] = d  # the timed kernel of this role is the one with the most dispatches
        else:
            if name in out["kernels"]:
                prev = out["kernels"].pop(name)
                out["kernels"][prev["kernel_name"]] = prev
            out["kernels"][name] = d
        d["kernel_name"] = k
    # the split coded launch (two shadow_coded kernels per batch: sphere tiles, raster-free
    # tiles): the shadow pass is both, so its per-launch counters and duration are the sums
    parts = {k: d for k, d in out["kernels"].items()
             if d.get("kernel_name", "").startswith("shadow_coded_batch_kernel<")}
    if len(parts) > 1:
        n = max(d["dispatches"] for d in parts.values())
        if all(d["dispatches"] >= 0.9 * n for d in parts.values()):
            merged = {"dispatches": n, "kernel_name": " + ".join(sorted(d["kernel_name"] for d in parts.values())),
                      "note": "split coded launch: the per-launch sums of its two kernels"}
            for c in set().union(*[set(d) for d in parts.values()]):
                if c in ("dispatches", "kernel_name", "hbm_bytes_note", "valu_insts_per_wave", "salu_insts_per_wave"):
                    continue
                if all(isinstance(d.get(c), (int, float)) for d in parts.values()):
                    merged[c] = sum(d[c] for d in parts.values())
            if merged.get("SQ_WAVES"):
                merged["valu_insts_per_wave"] = merged.get("SQ_INSTS_VALU", 0) / merged["SQ_WAVES"]
                merged["salu_insts_per_wave"] = merged.get("SQ_INSTS_SALU", 0) / merged["SQ_WAVES"]
            for k in list(parts):
                d = out["kernels"].pop(k)
                out["kernels"][d["kernel_name"]] = d
            out["kernels"]["shadow_pass"] = merged
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
