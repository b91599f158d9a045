"""Last steps of a rocprofv3 kernel trace as a timeline: kernel, start, duration (us)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40]
    print(f"{name:42s} start {(s - t0) / 1000:8.2f} dur {(e - s) / 1000:6.2f}")
