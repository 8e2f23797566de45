"""Per-kernel rocprofv3 durations of bench.py split into its passes.

bench.py (default arguments) dispatches every k_* kernel S times in the untimed
settle phase (config.settle.frames / config.frames_per_step of its line), W + K
times in the pipelined timed pass, W + K times in the roofline pass (one step at
a time, HIP events around each launch), then K times in the plain one-lane pass
(no events).  rocprofv3 --stats averages all of them;
this splits run_kernel_trace.csv by dispatch order so the roofline pass's
average can be compared with the `roofline.kernels[*].avg_launch_us` the bench
line reports for the same dispatches.
usage: kstats_passes.py <run_kernel_trace.csv> <out.csv> [W] [K] [S | bench line .json]
"""
import csv
import sys
from collections import defaultdict

trace, out = sys.argv[1], sys.argv[2]
W = int(sys.argv[3]) if len(sys.argv) > 3 else 20
K = int(sys.argv[4]) if len(sys.argv) > 4 else 200
S = 0
if len(sys.argv) > 5:
    a = sys.argv[5]
    if a.endswith(".json"):  # the bench line of the same run: its settle frame count
        import json
        cfg = json.load(open(a))["config"]  # (settle frames: launches x frames per step)
        S = int((cfg.get("settle") or {}).get("frames", 0)) // max(1, int(cfg.get("frames_per_step", 1)))
    else:
        S = int(a)
per = defaultdict(list)
for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Dispatch_Id"])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dmmt::", "").split("<")[0]
    if name in ("k_front", "k_hist", "k_tables", "k_emit", "k_offsets", "k_stuffwrite"):
        per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = []
for name, d in per.items():
    n = W + K
    passes = {"settle": d[:S], "timed_pipelined": d[S:S + n], "roofline_one_lane": d[S + n:S + 2 * n],
              "plain_one_lane": d[S + 2 * n:S + 2 * n + K], "all": d}
    for p, v in passes.items():
        if v:
            rows.append({"kernel": name, "pass": p, "dispatches": len(v), "avg_us": round(sum(v) / len(v), 2),
                         "min_us": round(min(v), 2), "max_us": round(max(v), 2)})
with open(out, "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0]))
    w.writeheader()
    w.writerows(rows)
for r in rows:
    print(f"{r['kernel']:14s} {r['pass']:18s} n={r['dispatches']:4d} avg_us={r['avg_us']:8.2f}")
