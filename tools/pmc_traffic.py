#!/usr/bin/env python3
"""Summarise a tools/pmc.sh run into profiles/: per-launch HBM traffic of k_march
(FETCH_SIZE + WRITE_SIZE, KB -> bytes) and the SQ counters, averaged over launches.
Usage: python tools/pmc_traffic.py <dir-glob> profiles/pmc_traffic.json [R S layout passes_per_launch]
(<dir-glob> matches the rocprofv3 output dirs, e.g. 'gpurun_out/pmc_*')."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    R, S, layout = (int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]) if len(sys.argv) > 5 else (512, 8, "corner8")
    F = int(sys.argv[6]) if len(sys.argv) > 6 else 16
    vals = defaultdict(list)
    for f in sorted(glob.glob(f"{src}/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "k_march" in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"kernel": "k_march", "resolution": R, "steps": S, "layout": layout,
           "passes_per_launch": F,
           "counters_mean_per_launch": mean,
           "note": "FETCH_SIZE/WRITE_SIZE in KB (rocprofv3); FETCH_SIZE is uncalibrated for "
                   "scattered 8-B gathers (MI355X_MICROARCH.md §HBM), reported uncorrected"}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        out["hbm_bytes_per_launch"] = int((mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out.get(k) for k in ("hbm_bytes_per_launch",)}))


if __name__ == "__main__":
    main()
