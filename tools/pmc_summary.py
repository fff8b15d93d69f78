#!/usr/bin/env python3
"""Average per-launch PMC counters of the march kernel from rocprofv3 csv dirs."""
import collections
import csv
import sys
from pathlib import Path

for d in sys.argv[1:]:
    for f in sorted(Path(d).glob("**/*counter_collection.csv")):
        agg = collections.defaultdict(float)
        n = collections.Counter()
        for r in csv.DictReader(open(f)):
            if "k_march" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
        out = {k: agg[k] / n[k] for k in agg}
        waves = out.get("SQ_WAVES")
        print(f.parent.name, {k: round(v) for k, v in out.items()})
        if waves:
            print("   per wave:", {k: round(v / waves, 1) for k, v in out.items() if k != "SQ_WAVES"})
