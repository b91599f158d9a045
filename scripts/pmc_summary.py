"""Per-kernel roofline table from rocprofv3 counter passes.

    python scripts/pmc_summary.py <counter_collection.csv> [...]

Each csv is one ``--pmc`` pass (scripts/gpu_run.sh ``pmc``: SQ set A, SQ set B, FETCH_SIZE,
WRITE_SIZE); the kernel-trace csv next to each one gives the dispatch durations.  Counters are
averaged per kernel over its dispatches, then combined:

  mfma%   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs): GRBM_GUI_ACTIVE
          reads ~8x the kernel cycles on MI355X (one count per XCD), the MFMA counter is per SIMD
  wait%   SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waves waiting on anything)
  winst%  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (waves waiting for an instruction's operands)
  ldsc%   SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  rdMB / wrMB   FETCH_SIZE / WRITE_SIZE (KB in the counters) per dispatch
  GB/s    (FETCH + WRITE) / mean kernel duration

Rows are sorted by total kernel time (calls x mean duration of the first pass that saw the kernel).
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.split("::")[-1][:44] if "<" not in n else n.split("::")[-1][:44]


def durations(counter_csv: str) -> dict:
    """{kernel: [duration_us, ...]} from the kernel-trace csv of the same run directory."""
    out = defaultdict(list)
    for path in glob.glob(os.path.join(os.path.dirname(counter_csv), "*kernel_trace.csv")):
        for r in csv.DictReader(open(path)):
            try:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            except (KeyError, ValueError):
                continue
            out[short(r["Kernel_Name"])].append(d)
    return out


def main(paths):
    cnt = defaultdict(lambda: defaultdict(list))
    dur = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in durations(p).items():
            dur.setdefault(k, v)
    rows = []
    for k, cs in cnt.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dur.get(k, [])
        us = sum(d) / len(d) if d else float("nan")
        rows.append((len(d) * us if d else 0.0, k, len(d), us, avg))
    rows.sort(key=lambda t: -t[0])
    total = sum(t[0] for t in rows) or 1.0
    print(f"{'kernel':44s} {'calls':>5s} {'us':>8s} {'%time':>6s} {'mfma%':>6s} {'wait%':>6s} {'winst%':>6s} "
          f"{'ldsc%':>6s} {'rdMB':>8s} {'wrMB':>8s} {'GB/s':>7s}")

    def pct(a, b):
        return 100.0 * a / b if a is not None and b else float("nan")

    for tot, k, n, us, a in rows:
        mfma = pct(a.get("SQ_VALU_MFMA_BUSY_CYCLES"), a.get("GRBM_GUI_ACTIVE", 0) / XCDS * CUS * SIMDS)
        wait = pct(a.get("SQ_WAIT_ANY"), a.get("SQ_WAVE_CYCLES"))
        winst = pct(a.get("SQ_WAIT_INST_ANY"), a.get("SQ_WAVE_CYCLES"))
        ldsc = pct(a.get("SQ_LDS_BANK_CONFLICT"), a.get("SQ_ACTIVE_INST_LDS"))
        rd = a.get("FETCH_SIZE", float("nan")) / 1024.0
        wr = a.get("WRITE_SIZE", float("nan")) / 1024.0
        moved = (rd if rd == rd else 0.0) + (wr if wr == wr else 0.0)
        gbs = moved * 1e3 / us if (rd == rd or wr == wr) and us == us and us > 0 else float("nan")  # MB/us -> GB/s
        print(f"{k:44s} {n:5d} {us:8.2f} {100 * tot / total:6.2f} {mfma:6.1f} {wait:6.1f} {winst:6.1f} "
              f"{ldsc:6.1f} {rd:8.2f} {wr:8.2f} {gbs:7.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
