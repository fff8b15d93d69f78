#!/usr/bin/env python3
"""Split the wall time of bench.py's timed region against the kernel (VERDICT
r03 weak 3 / next 6): where the microseconds between the host's clock around
the region and the march kernel's own duration go.

Inputs: the host clocks bench.py writes with VPTMCM_BENCH_STAMPS=<json>
(CLOCK_MONOTONIC and CLOCK_BOOTTIME just before the region's perf_counter
start and just after its end, plus the enqueue return) and the rocprofv3
kernel trace of the same run (--kernel-trace, csv). rocprofv3's timestamps are
host-clock nanoseconds; the clock whose window contains the region's kernels
is used.

    python tools/wall_split.py <stamps.json> <kernel_trace.csv>
"""
import csv
import json
import sys


def main():
    st = json.load(open(sys.argv[1]))
    rows = list(csv.DictReader(open(sys.argv[2])))
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    out = None
    for clock in ("monotonic_ns", "boottime_ns"):
        a, b = st[clock]
        inside = sorted(k for k in kern if a <= k[0] and k[1] <= b)
        if inside:
            out = (clock, a, b, inside)
            break
    if out is None:
        raise SystemExit("no kernel of the trace lies inside the region on either clock")
    clock, a, b, inside = out
    # a and b bracket the perf_counter region within a few hundred ns (the
    # clock_gettime calls next to it); perf_counter offsets place t0 / t_enq
    wall_us = st["el_s"] * 1e6
    t0 = a  # <= the region's start
    enq_us = (st["t_enq_perf"] - st["t0_perf"]) * 1e6
    first, last = inside[0], inside[-1]
    res = {
        "clock": clock,
        "kernels": [k[2][:60] for k in inside],
        "wall_us": round(wall_us, 2),
        "bracket_us": round((b - a) / 1e3, 2),
        "enqueue_return_us": round(enq_us, 2),
        "start_to_first_kernel_us": round((first[0] - t0) / 1e3, 2),
        "kernel_span_us": round((last[1] - first[0]) / 1e3, 2),
        "kernel_busy_us": round(sum(k[1] - k[0] for k in inside) / 1e3, 2),
        "last_kernel_end_to_region_end_us": round((b - last[1]) / 1e3, 2),
    }
    res["wall_minus_kernel_us"] = round(wall_us - res["kernel_span_us"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
