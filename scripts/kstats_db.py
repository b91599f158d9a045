"""Summarise a rocprofv3 SQLite result (run_results.db, the default output format): per kernel
calls, average and total time, share of the traced kernel time; optional per-step division."""
import sqlite3
import sys

db = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration), sum(duration) from kernels group by name").fetchall()
tot = sum(r[3] for r in rows)
for name, n, avg, s in sorted(rows, key=lambda r: -r[3]):
    per = f" per_step_us={s / steps / 1e3:8.2f}" if steps else ""
    print(f"{name[:90]:90s} calls={n:>6} avg_us={avg / 1e3:8.2f}{per} pct={100 * s / tot:6.2f}")
print("total kernel ms", round(tot / 1e6, 3), ("per step us %.1f" % (tot / steps / 1e3)) if steps else "")
