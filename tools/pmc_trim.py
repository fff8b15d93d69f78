#!/usr/bin/env python3
"""Trim rocprofv3 counter passes to the rows of their last measured dispatch.

    python tools/pmc_trim.py gpurun_out/pmcreq profiles/rNN/pmcreq

Every <pass>/run_counter_collection.csv under the source becomes <pass>.csv in
the destination, keeping the header and the rows of the last dispatch of the
march (k_march) or of the known-bytes gather (k_gather) — the inputs
tools/pmc_report.py reads.
"""
import csv
import sys
from pathlib import Path


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    for d in sorted(p for p in src.iterdir() if p.is_dir()):
        f = d / "run_counter_collection.csv"
        if not f.exists():
            continue
        rows = list(csv.DictReader(open(f)))
        keep = [r for r in rows if "k_march" in r["Kernel_Name"] or "gather" in r["Kernel_Name"]]
        if not keep:
            continue
        last = max(int(r["Dispatch_Id"]) for r in keep)
        out = [r for r in keep if int(r["Dispatch_Id"]) == last]
        with open(dst / f"{d.name}.csv", "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(out)
        print(d.name, len(out))


if __name__ == "__main__":
    main()
