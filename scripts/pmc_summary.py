"""Average rocprofv3 PMC counters per kernel over its dispatches.
usage: pmc_summary.py <dir with p*/run_counter_collection.csv> [name filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "**", "run_counter_collection.csv"), recursive=True)):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if flt not in name:
            continue
        per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, d, c), v in per.items():
        acc[name][c].append(v)
for name, cs in acc.items():
    print(name[:70])
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} {sum(vs)/len(vs):16.1f}  (n={len(vs)})")
