"""Concurrency of the pipelined lanes from a rocprofv3 --kernel-trace CSV: per
kernel the summed busy time, and the wall time split by how many kernels run at
once.  usage: timeline.py run_kernel_trace.csv [n_dispatches] [skip]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = [r for r in rows if "dmmt::k_" in r["Kernel_Name"] and "synthetic" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[skip:skip + n]
ev = []
busy = defaultdict(float)
for r in rows:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dmmt::", "").split("<")[0]
    busy[k] += (b - a) / 1e3
    ev += [(a, 1, k), (b, -1, k)]
ev.sort()
t0, t1 = ev[0][0], ev[-1][0]
conc = defaultdict(float)
active = defaultdict(int)
last = t0
for t, d, k in ev:
    nact = sum(active.values())
    conc[nact] += (t - last) / 1e3
    last = t
    active[k] += d
wall = (t1 - t0) / 1e3
fronts = sum(1 for r in rows if "k_front" in r["Kernel_Name"])
print(f"window {wall:.1f} us, {fronts} frames, {wall / max(fronts, 1):.2f} us/frame")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {k:14s} busy {v / max(fronts, 1):7.2f} us/frame")
for c in sorted(conc):
    print(f"  {c} kernels running: {100 * conc[c] / wall:5.1f} % of wall")
