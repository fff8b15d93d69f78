#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace's k_march dispatches into the bench's launch
kinds (fused multi-pass launches vs one-pass launches) so the per-launch
average can be compared with bench.py's event-timed kernel_avg_us.
Usage: python tools/trace_split.py run_kernel_trace.csv [out.json [W K F [SETTLE]]]
(SETTLE = config.clock_settle_passes of the profiled bench line: untimed
clock-settling launches of F passes that precede the warm-up)"""
import csv
import json
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_march<" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    # bench order: 1 warm-up launch (16 passes), K/16 timed fused launches, then
    # the one-pass launches of the unfused region
    long_ = [x for x in d if x > 100.0]
    short = [x for x in d if x <= 100.0]
    # bench order: warm-up launches, timed launches, one-pass launches, then the
    # render_api launches; counts from the bench defaults unless given
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    F = int(sys.argv[5]) if len(sys.argv) > 5 else 32
    settle = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    warm, timed = settle // F + -(-W // F), -(-K // F)
    t = long_[warm:warm + timed]
    api = long_[warm + timed:]
    out = {"k_march_dispatches": len(d),
           "fused_launches": {"n": len(long_), "avg_us": round(sum(long_) / max(1, len(long_)), 3),
                              "timed_region_avg_us": round(sum(t) / max(1, len(t)), 3),
                              "timed_region_n": len(t),
                              "render_api_avg_us": round(sum(api) / max(1, len(api)), 3) if api else None},
           "one_pass_launches": {"n": len(short), "avg_us": round(sum(short) / max(1, len(short)), 3)}}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
