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
    chains, packs, comps, gaps, pack_chain, march_gap = [], [], [], [], [], []
    group = []

    def close(g):
        marches = [x for x in g if x[0] == "march"]
        pk = [x for x in g if x[0] == "pack"]
        cm = [x for x in g if x[0] == "composite"]
        if not (marches and cm):
            return
        last_march = max(x[2] for x in marches)
        chains.append((max(x[2] for x in cm) - last_march) / 1e3)
        packs.extend((x[2] - x[1]) / 1e3 for x in pk)
        comps.extend((x[2] - x[1]) / 1e3 for x in cm)
        march_gap.append((min(x[1] for x in cm) - last_march) / 1e3)
        if pk:  # the cross-stream wait: last pack done -> first shard kernel starts
            gaps.append((min(x[1] for x in cm) - max(x[2] for x in pk)) / 1e3)
            pack_chain.append((max(x[2] for x in pk) - last_march) / 1e3)

    for x in kinds:  # a region: marches, then its packs and composites
        if x[0] == "march" and any(g[0] == "composite" for g in group):
            close(group)
            group = []
        group.append(x)
    close(group)
    med = lambda v: round(statistics.median(v), 2) if v else None
    print(json.dumps({"composites": len(chains), "chain_us_median": med(chains),
                      "chain_us_p90": round(sorted(chains)[int(0.9 * len(chains))], 2) if chains else None,
                      "last_march_to_first_shard_us_median": med(march_gap),
                      "last_march_to_last_pack_us_median": med(pack_chain),
                      "last_pack_to_first_shard_us_median": med(gaps),
                      "k_pack_us_median": med(packs), "k_composite_us_median": med(comps)}))


if __name__ == "__main__":
    main()
