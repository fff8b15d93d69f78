#!/usr/bin/env python3
"""profiles/pmc_traffic.json from the tools/pmc_req.sh passes (measurement aid).

Memory-side read bytes are counted from the L2's fabric read requests BY SIZE
(TCC_EA0_RDREQ_32B/_64B/_128B): no FETCH_SIZE factor is needed. The known-bytes
gather launch (tools/gather_calib: scattered 8-B loads, count known) shows what
one march gather costs: one 128-B request per gather, and FETCH_SIZE = requests
x 64 B (so the guide's gfx950 x2 FETCH_SIZE correction holds for gathers too).
Write bytes: WRITE_SIZE (the r01 known-bytes launch calibrated it at 0.997).

Issue fields (SQ pass): VALU / SALU wave-instructions per launch, the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration) and the chip-wide VALU issue
fraction: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles
(MI355X_MICROARCH.md, wave scheduling), so 1024 SIMDs issue at most
512 wave-instructions per cycle.

Usage: python tools/pmc_report.py <pmcreq dir> <out.json> [R S layout volume [camera]]
(<pmcreq dir>: gpurun_out/pmcreq as rocprofv3 wrote it, or profiles/r02/pmcreq
with one trimmed <pass>.csv per counter pass)
"""
import csv
import json
import re
import sys
from pathlib import Path

SIMDS = 1024


def last_dispatch(d: Path, kernel: str):
    """Counters (summed over rows) and duration of the last dispatch of `kernel`."""
    f = d / "run_counter_collection.csv" if d.is_dir() else d.with_name(d.name + ".csv")
    rows = list(csv.DictReader(open(f)))
    ids = [int(r["Dispatch_Id"]) for r in rows if kernel in r["Kernel_Name"]]
    if not ids:
        raise SystemExit(f"no {kernel} dispatch under {d}")
    last = max(ids)
    c, dur = {}, None
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            name = r["Kernel_Name"]
    return c, dur, name


def read_bytes(c):
    return 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + \
        128 * c["TCC_EA0_RDREQ_128B_sum"]


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    R, S, layout, volume, camera = 512, 8, "corner8", 512, "default"
    if len(sys.argv) > 6:
        R, S, layout, volume = int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6])
    if len(sys.argv) > 7:
        camera = sys.argv[7]
    out = {"source": "tools/pmc_req.sh + tools/pmc_report.py", "entries": []}

    gathers = 4096 * 256 * 256  # tools/gather_calib defaults: 4096 blocks x 256 lanes x 256
    if (src / "calib_req").exists() or (src / "calib_req.csv").exists():
        cq, cdur, _ = last_dispatch(src / "calib_req", "k_gather")
        cf, _, _ = last_dispatch(src / "calib_fetch", "k_gather")
        out["gather_calibration"] = {
            "launch": "tools/gather_calib 1024: 268,435,456 scattered 8-B loads from a 1 GiB table",
            "requests_per_gather": round(cq["TCC_EA0_RDREQ_sum"] / gathers, 4),
            "req_128B_share": round(cq["TCC_EA0_RDREQ_128B_sum"] / cq["TCC_EA0_RDREQ_sum"], 5),
            "read_bytes_per_gather": round(read_bytes(cq) / gathers, 2),
            "fetch_size_bytes_per_gather": round(cf["FETCH_SIZE"] * 1024 / gathers, 2),
            "fetch_size_factor": round(read_bytes(cq) / (cf["FETCH_SIZE"] * 1024), 4),
            "gathers_per_s_under_pmc": round(gathers / cdur, 1),
        }
    elif dst.exists():  # passes of another camera / volume: the file's calibration stands
        out["gather_calibration"] = json.loads(dst.read_text()).get("gather_calibration")
    for ppl_dir in sorted({p.with_suffix("") for p in src.glob("bench*_req*")}):
        ppl = int(ppl_dir.name[len("bench"):-len("_req")])
        q, qdur, kname = last_dispatch(ppl_dir, "k_march")
        wd = src / f"bench{ppl}_write"
        w = last_dispatch(wd, "k_march")[0] if wd.exists() or wd.with_name(wd.name + ".csv").exists() \
            else {"WRITE_SIZE": 0.0}  # no write pass: reads only
        sq, sdur, _ = last_dispatch(src / f"bench{ppl}_sq", "k_march")
        rb = read_bytes(q)
        wb = w["WRITE_SIZE"] * 1024
        cycles = sq["GRBM_GUI_ACTIVE"] / 8
        valu, salu = sq["SQ_INSTS_VALU"], sq["SQ_INSTS_SALU"]
        photon_steps = R * R * S * ppl
        # k_march<L, SPEC, MODE, MAJ>: the macro-cell bound is the 4th template
        # argument (rocprofv3 writes the demangled name)
        mj = re.search(r"k_march<\d+u, (?:true|false), \d+u, (true|false)>", kname)
        out["entries"].append({
            "kernel": "k_march", "kernel_name": kname, "resolution": R, "steps": S, "layout": layout,
            "volume": volume, "passes_per_launch": ppl, "camera": camera,
            "macro_skip": bool(mj and mj.group(1) == "true"),
            "kernel_us_under_pmc": round(qdur * 1e6, 2),
            "read_requests": {"32B": q["TCC_EA0_RDREQ_32B_sum"], "64B": q["TCC_EA0_RDREQ_64B_sum"],
                              "128B": q["TCC_EA0_RDREQ_128B_sum"]},
            "read_bytes_per_launch": int(rb), "write_bytes_per_launch": int(wb),
            "hbm_bytes_per_launch": int(rb + wb),
            "memory_side_tbps_under_pmc": round((rb + wb) / qdur * 1e-12, 3),
            "issue": {
                "valu_insts": valu, "salu_insts": salu,
                "valu_trans_f32": sq["SQ_INSTS_VALU_TRANS_F32"],
                "valu_per_photon_step": round(valu * 64 / photon_steps, 2),
                "waves": sq["SQ_WAVES"], "effective_ghz": round(cycles / sdur * 1e-9, 3),
                "valu_issue_frac": round(valu * 2 / (SIMDS * cycles), 4),
                "note": "chip-wide: VALU wave-instructions x 2 cycles / (1024 SIMDs x kernel cycles)",
            },
        })
    if dst.exists():  # keep the file's other top-level fields (gather_peak, ...)
        for k, v in json.loads(dst.read_text()).items():
            out.setdefault(k, v)
    if dst.exists():  # keep the other layouts' / shapes' entries
        key = lambda e: (e["resolution"], e["steps"], e["layout"], e["volume"], e["passes_per_launch"],
                         e.get("camera", "default"), e.get("macro_skip", False))
        mine = {key(e) for e in out["entries"]}
        old = json.loads(dst.read_text()).get("entries", [])
        out["entries"] = [e for e in old if key(e) not in mine] + out["entries"]
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out["gather_calibration"]))
    for e in out["entries"]:
        print(e["passes_per_launch"], e["hbm_bytes_per_launch"], e["issue"]["valu_issue_frac"],
              e["issue"]["valu_per_photon_step"], e["issue"]["effective_ghz"])


if __name__ == "__main__":
    main()
