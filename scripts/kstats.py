"""Summarise a rocprofv3 kernel_stats.csv (and per-step time from the kernel trace)."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    per = f' per_step_us={float(r["TotalDurationNs"]) / steps / 1e3:8.2f}' if steps else ""
    print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>6} avg_us={float(r["AverageNs"]) / 1e3:8.2f}{per} pct={float(r["Percentage"]):6.2f}')
print("total kernel ms", round(tot / 1e6, 3), ("per step us %.1f" % (tot / steps / 1e3)) if steps else "")
