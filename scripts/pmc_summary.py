#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/<variant>_g<k>/run_counter_collection.csv)
into per-kernel mean counter values per launch, and HBM traffic per launch as
FETCH_SIZE*2 + WRITE_SIZE (KB -> bytes; MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the
bytes of wide coalesced streams)."""
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


def main(root, out, config):
    res = defaultdict(lambda: defaultdict(list))
    for d in sorted(glob.glob(os.path.join(root, "*_g*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        var = os.path.basename(d).split("_")[0]
        for r in csv.DictReader(open(f)):
            k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sph::", ""))
            res[(var, k)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    summary = {}
    for (var, k), cs in sorted(res.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        summary.setdefault(var, {})[k] = m
    A = GE.load_package()._abi
    # the kernels these counters belong to: bench.py uses the file only for the same code objects
    doc = {"config": config, "source": "rocprofv3 --kernel-trace --pmc, one counter group per run",
           "device_code_hash": A.device_code_hash(), "lib": str(A.lib_path().name), "kernels": summary}
    force = {}
    for var, ks in summary.items():
        for k in ("k_force_tiled", "k_force_integrate"):
            if k in ks and "hbm_bytes_per_launch" in ks[k]:
                force[var] = ks[k]["hbm_bytes_per_launch"]
    # bench.py reads kernel_bytes.force_integrate for the default variant
    default = "1"
    if f"v{default}" in force:
        doc["kernel_bytes"] = {"force_integrate": force[f"v{default}"]}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({v: {k: {c: round(x, 1) for c, x in m.items() if c in ("hbm_bytes_per_launch", "SQ_INSTS_VALU",
                                                                              "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")}
                          for k, m in ks.items() if k.startswith("k_")} for v, ks in summary.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "C3")
