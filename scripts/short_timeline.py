"""Fill and drain of a short pipelined run from a rocprofv3 --kernel-trace CSV of
scripts/short_probe.py: the last `frames` frames (6 launches each), per frame its
lane (stream), start of k_front, end of k_stuffwrite and latency, relative to the
first k_front.  usage: short_timeline.py run_kernel_trace.csv [frames]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "dmmt::k_" in r["Kernel_Name"]]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20


def short(name):
    return name.split("(")[0].replace("void ", "").replace("dmmt::", "").split("<")[0]


rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if short(r["Kernel_Name"]) != "k_synthetic"]
rows = rows[-6 * frames:]
# a frame = a k_front and the next five launches on its stream
streams = {}
out = []
for r in rows:
    s = r.get("Stream_Id") or r.get("Queue_Id")
    k = short(r["Kernel_Name"])
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if k == "k_front":
        streams[s] = {"stream": s, "front0": a, "kern": {}}
        out.append(streams[s])
    if s in streams:
        streams[s]["kern"][k] = (a, b)
t0 = min(f["front0"] for f in out)
tend = max(max(b for _, b in f["kern"].values()) for f in out)
print(f"frames={len(out)} first k_front -> last end = {(tend - t0) / 1e3:.1f} us "
      f"({(tend - t0) / 1e3 / len(out):.1f} us/frame)")
for i, f in enumerate(out):
    end = max(b for _, b in f["kern"].values())
    parts = " ".join(f"{k[2:]}={(b - a) / 1e3:.1f}" for k, (a, b) in sorted(f["kern"].items(), key=lambda x: x[1][0]))
    print(f"{i:2d} stream={f['stream']} start={(f['front0'] - t0) / 1e3:7.1f} end={(end - t0) / 1e3:7.1f} "
          f"latency={(end - f['front0']) / 1e3:6.1f}  {parts}")
