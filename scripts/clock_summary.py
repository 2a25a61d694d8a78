#!/usr/bin/env python3
"""Effective shader clock per kernel from rocprofv3 passes with `--kernel-trace --pmc GRBM_GUI_ACTIVE
GRBM_COUNT`: clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS give-back;
the quotient reads high on dispatches shorter than ~0.3 ms, so long dispatches are the measurement).
Dispatches shorter than MIN_US are dropped: the GRBM count of a short dispatch includes its launch ramp and
reads 3-17 GHz (profiles/clock_r03.json), which no clock reaches. A `valu_peak=<log>` argument adds the VALU
microbenchmark's issue rate measured in the same run on the same box (scripts/valu_peak.hip JSON lines; the
8-waves-per-SIMD plain-f32 line), so the rate and its clock come from one box.
Usage: clock_summary.py <out.json> <label>=<rocprof dir> ... [valu_peak=<log>]"""
import re
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402


MIN_US = 50.0


def one(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        return {"error": f"missing csv in {d}: {cc} {kt}"}
    dur = {}
    rows = list(csv.DictReader(open(kt[0])))
    for r in rows:
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[key] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(lambda: defaultdict(list))
    crow = list(csv.DictReader(open(cc[0])))
    for r in crow:
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sph::", ""))
        per[k][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
    out = {"columns_counter": list(crow[0].keys()) if crow else [], "columns_trace": list(rows[0].keys()) if rows else []}
    for k, cs in per.items():
        g = dict(cs.get("GRBM_GUI_ACTIVE", []))
        clocks, durs = [], []
        for key, v in g.items():
            if key in dur and dur[key] > 0:
                clocks.append(v / 8.0 / dur[key] / 1e9)
                durs.append(dur[key] * 1e6)
        keep = [(c, u) for c, u in zip(clocks, durs) if u >= MIN_US]
        if clocks and not keep:
            out[k] = {"dispatches": len(clocks), "mean_us": sum(durs) / len(durs),
                      "dropped": f"every dispatch shorter than {MIN_US:g} us: no clock reading"}
            continue
        clocks, durs = [c for c, _ in keep], [u for _, u in keep]
        if clocks:
            clocks.sort()
            out[k] = {"dispatches": len(clocks), "mean_us": sum(durs) / len(durs),
                      "clock_ghz_median": clocks[len(clocks) // 2], "clock_ghz_min": clocks[0], "clock_ghz_max": clocks[-1]}
    return out


def main():
    res = {"method": "GRBM_GUI_ACTIVE / 8 / kernel duration, rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT",
           "device_code_hash": GE.load_package()._abi.device_code_hash()}
    for arg in sys.argv[2:]:
        label, d = arg.split("=", 1)
        if label == "valu_peak":
            rows = [json.loads(l) for l in open(d) if l.startswith("{")]
            best = [r for r in rows if r.get("waves_per_simd") == 8 and r.get("packed") == 0]
            res[label] = {"file": os.path.basename(d), **(best[0] if best else {"error": "no 8-wave plain line"})}
            continue
        res[label] = one(d)
    json.dump(res, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
