"""Per-kernel time of the last K steps in a rocprofv3 kernel trace: launches, summed duration per
step, and the idle time between consecutive dispatches (the step's wall span minus busy time, where dispatches of
several streams may overlap). usage: trace_window.py run_kernel_trace.csv STEPS_TIMED STEP_MARKER_KERNEL"""
import csv
import re
import sys
from collections import defaultdict

f, steps, marker = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader(open(f)))
ev = []
for r in rows:
    k = re.sub(r"<[^>]*>", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sph::", "")).strip()
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
ev.sort()
# the last `steps` steps: from the steps-th last dispatch of the marker kernel on
starts = [i for i, e in enumerate(ev) if e[2] == marker]
first = starts[-steps]
win = ev[first:]
t0, t1 = win[0][0], max(e[1] for e in win)
per = defaultdict(lambda: [0, 0])
for s, e, k in win:
    per[k][0] += 1
    per[k][1] += e - s
busy, cur_s, cur_e = 0, None, None
for s, e, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = (t1 - t0) / steps / 1e3
print(f"steps {steps}: span {span:.1f} us/step, busy (union of dispatches) {busy / steps / 1e3:.1f} us/step, "
      f"idle {span - busy / steps / 1e3:.1f} us/step, launches {len(win) / steps:.1f}/step")
for k, (n, d) in sorted(per.items(), key=lambda x: -x[1][1]):
    print(f"  {k:40s} {n / steps:6.2f}/step  {d / steps / 1e3:8.1f} us/step  {d / n / 1e3:7.1f} us each")
