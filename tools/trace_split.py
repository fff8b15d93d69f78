#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace's k_march dispatches into the bench's launch
kinds (fused multi-pass launches vs one-pass launches) so the per-launch
average can be compared with bench.py's event-timed kernel_avg_us.
Usage: python tools/trace_split.py run_kernel_trace.csv [out.json]"""
import csv
import json
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_march" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    # bench order: 1 warm-up launch (16 passes), K/16 timed fused launches, then
    # the one-pass launches of the unfused region
    long_ = [x for x in d if x > 100.0]
    short = [x for x in d if x <= 100.0]
    out = {"k_march_dispatches": len(d),
           "fused_launches": {"n": len(long_), "avg_us": round(sum(long_) / max(1, len(long_)), 3),
                              "timed_avg_us (excl. warm-up)": round(sum(long_[1:]) / max(1, len(long_) - 1), 3)},
           "one_pass_launches": {"n": len(short), "avg_us": round(sum(short) / max(1, len(short)), 3)}}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
