"""Per-launch HBM traffic of every kernel from scripts/gpu_traffic.sh passes.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts
half the bytes of wide (16 B/lane) streaming reads (MI355X_MICROARCH.md, HBM
section), so it is doubled here (every hot kernel of this path reads with
16-byte loads).  Writes the JSON bench.py reads for roofline.traffic.
usage: pmc_json.py <pmc dir> <out.json> [config]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
config = sys.argv[3] if len(sys.argv) > 3 else "4k444q90"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, _, c), v in per.items():
        acc[name][c].append(v)


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("dmmt::", "")
    return n.split("<")[0]


kernels = {}
for name, cs in acc.items():
    k = short(name)
    if not k.startswith("k_"):
        continue
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {"dispatches": max(len(v) for v in cs.values())}
    if "FETCH_SIZE" in d:
        e["fetch_bytes_raw"] = d["FETCH_SIZE"] * 1024
        e["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in d:
        e["write_bytes"] = d["WRITE_SIZE"] * 1024
    if "fetch_bytes" in e and "write_bytes" in e:
        e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
    for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
              "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
        if c in d:
            e[c] = d[c]
    kernels[k] = e
res = {"config": config, "source": os.path.abspath(root), "note": __doc__.strip().splitlines()[0],
       "kernels": kernels,
       "front_hbm_bytes_per_launch": kernels.get("k_front", {}).get("hbm_bytes")}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {kk: round(vv) for kk, vv in v.items() if "bytes" in kk} for k, v in kernels.items()}, indent=1))
