"""Gaps between consecutive kernels in a rocprofv3 kernel trace (CSV): which kernel precedes the idle
time, on average, over the last N dispatches. Usage: trace_gaps.py run_kernel_trace.csv [N]"""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
gap = defaultdict(list)
busy = 0
for a, b in zip(rows, rows[1:]):
    name = a["Kernel_Name"].split("(")[0].replace("void ", "")
    gap[name].append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
for r in rows:
    busy += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"dispatches {len(rows)} span {span/1e3:.1f} us busy {busy/1e3:.1f} us ({busy/span:.3f})")
for k, v in sorted(gap.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k[:60]:60s} n {len(v):5d} mean gap {sum(v)/len(v)/1e3:7.2f} us  median {v[len(v)//2]/1e3:7.2f}  total {sum(v)/1e3:9.1f} us")
