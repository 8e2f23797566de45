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
# pairwise: wall time during which both kernels of a pair are running
iv = defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dmmt::", "").split("<")[0]
    iv[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))


def union(xs):
    xs = sorted(xs)
    out = []
    for a, b in xs:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


U = {k: union(v) for k, v in iv.items()}
for k in sorted(U):
    cov = sum(b - a for a, b in U[k]) / 1e3
    print(f"  {k:14s} covers {100 * cov / wall:5.1f} % of wall")
ks = sorted(U)
for i in range(len(ks)):
    for j in range(i + 1, len(ks)):
        o = overlap(U[ks[i]], U[ks[j]]) / 1e3
        if o > 0.02 * wall:
            print(f"  {ks[i]} & {ks[j]} overlap {100 * o / wall:5.1f} % of wall")
