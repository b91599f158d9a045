"""Average rocprofv3 --pmc counter values per kernel (one row per dispatch x counter)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0].split("::")[-1][:40]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    line = " ".join(f"{c}={sum(v) / len(v):.3g}" for c, v in sorted(cs.items()))
    print(f"{k:40s} {line}")
