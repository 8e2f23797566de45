# time to idle of N pipelined frames (4 lanes) for small N: the fill/drain curve
set -o pipefail
mkdir -p gpurun_out/fill
for n in 1 2 3 4 6 8 12 20 40; do
  timeout -k 10 120 python scripts/short_probe.py --steps $n --runs 6 > gpurun_out/fill/n$n.txt 2>&1 || { echo "probe $n failed"; tail gpurun_out/fill/n$n.txt; exit 1; }
  python - "$n" <<'PY'
import re, sys
n = sys.argv[1]
v = [float(m.group(1)) for m in re.finditer(r"idle_at=(\d+)us", open(f"gpurun_out/fill/n{n}.txt").read())][1:]
e = [float(m.group(1)) for m in re.finditer(r"enqueue=(\d+)us", open(f"gpurun_out/fill/n{n}.txt").read())][1:]
print(f"N={n} idle_at median={sorted(v)[len(v)//2]:.0f}us min={min(v):.0f} enqueue median={sorted(e)[len(e)//2]:.0f}us")
PY
done
echo exit=0
