"""Print a rocprofv3 kernel_stats.csv as a compact table."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:48]:48s} calls={int(r['Calls']):>6} avg_us={float(r['AverageNs'])/1000:9.2f} "
          f"min_us={float(r['MinNs'])/1000:8.2f} total_ms={float(r['TotalDurationNs'])/1e6:8.2f} pct={float(r['Percentage']):6.2f}")
