#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of scripts/profile.sh into profiles/.

Reads the kernel-trace stats and the --pmc counter CSVs of one profiling
call and writes a JSON summary with per-launch averages for the SHA-256 and
Base64 kernels:
  * kernel durations (kernel-trace stats)
  * HBM traffic per launch: FETCH_SIZE x 2 (gfx950 reports half the bytes of
    a wide coalesced read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, in bytes
  * VALU instruction counts and the effective clock (GRBM_GUI_ACTIVE / 8 /
    kernel time).
Usage: tools/pmc_summary.py <prof_dir> <out_json> <workload-tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {"sha256_b64dec": "sha_b64dec", "sha256_lanes": "sha", "b64_encode_kernel": "b64enc", "b64_decode_kernel": "b64dec",
           "gather_kernel": "gather", "synth_kernel": "synth"}


def short(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def read_rows(pattern):
    rows = []
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main():
    prof, out, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    summary = {"workload": tag, "source": os.path.relpath(prof), "kernels": {}}
    # durations
    for r in read_rows(os.path.join(prof, "**", "*kernel_stats.csv")):
        k = short(r["Name"])
        if k:
            summary["kernels"].setdefault(k, {})["avg_ms"] = float(r["AverageNs"]) / 1e6
            summary["kernels"][k]["calls"] = int(r["Calls"])
    # counters: average per dispatch, per kernel
    acc = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for r in read_rows(os.path.join(prof, "**", "*counter_collection.csv")):
        k = short(r.get("Kernel_Name", ""))
        if not k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            durs[(k, r.get("Dispatch_Id"))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    for k, ctrs in acc.items():
        d = summary["kernels"].setdefault(k, {})
        for name, vals in ctrs.items():
            d[name] = sum(vals) / len(vals)
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = 2.0 * d["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024.0
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        kd = [v for (kk, _), v in durs.items() if kk == k]
        if kd:
            d["pmc_dispatch_s"] = sum(kd) / len(kd)
            if "GRBM_GUI_ACTIVE" in d:
                d["effective_clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8.0 / d["pmc_dispatch_s"] / 1e9
    sha = summary["kernels"].get("sha", {})
    summary["sha_hbm_bytes_per_launch"] = sha.get("hbm_bytes")
    summary["b64_hbm_bytes_per_launch"] = summary["kernels"].get("b64enc", {}).get("hbm_bytes")
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
