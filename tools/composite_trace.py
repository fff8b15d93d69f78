#!/usr/bin/env python3
"""Device chain of the device-list composite from a rocprofv3 kernel trace of
tools/group_enqueue.py --composite (measurement aid).

For every composite (one per render_passes call): from the end of the last
k_march of the region to the end of the last k_composite of it, and the
k_pack / k_composite durations. With the replicas on one GPU the marches
serialise and every shard kernel runs on that GPU, so the chain is an upper
bound on the device part of an N-GPU composite except for its xGMI transfer
(which is not measured here: one GPU per builder box).

    python tools/composite_trace.py <run_kernel_trace.csv>
"""
import csv
import json
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    kinds = []
    for r in rows:
        name = r["Kernel_Name"]
        k = "march" if "k_march" in name else "pack" if "k_pack" in name else \
            "composite" if "k_composite" in name else None
        if k:
            kinds.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    chains, packs, comps = [], [], []
    last_march, comp_end, seen = None, None, False
    for k, b, e in kinds:
        if k == "march":
            if seen:  # the previous region's composite is complete: a new region
                chains.append((comp_end - last_march) / 1e3)
                seen, last_march = False, None
            last_march = e if last_march is None else max(last_march, e)
        elif k == "pack":
            packs.append((e - b) / 1e3)
        else:
            comps.append((e - b) / 1e3)
            comp_end = e if not seen else max(comp_end, e)
            seen = True
    if seen:
        chains.append((comp_end - last_march) / 1e3)
    med = lambda v: round(statistics.median(v), 2) if v else None
    print(json.dumps({"composites": len(chains), "chain_us_median": med(chains),
                      "chain_us_p90": round(sorted(chains)[int(0.9 * len(chains))], 2) if chains else None,
                      "k_pack_us_median": med(packs), "k_composite_us_median": med(comps)}))


if __name__ == "__main__":
    main()
