"""Per-kernel mean duration over the last N dispatches of a rocprofv3 kernel trace (CSV), e.g. the
mid-collapse section at the end of a bench run. Usage: trace_kstats.py run_kernel_trace.csv [N]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"dispatches {len(rows)} span {span / 1e3:.1f} us")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:50]:50s} n {len(v):5d} mean {sum(v) / len(v) / 1e3:8.2f} us  max {max(v) / 1e3:8.2f} us  "
          f"total {sum(v) / 1e3:10.1f} us")
