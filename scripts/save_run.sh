#!/bin/bash
# Copy a finished gpurun's logs (and kernel-stats summaries) from gpurun_out/ into profiles/<dest>/
set -eu
dest="profiles/$1"
mkdir -p "$dest"
cp gpurun_out/*.log "$dest"/ 2>/dev/null || true
for d in gpurun_out/*/; do
  [ -f "$d/run_kernel_stats.csv" ] && python scripts/kstats.py "$d/run_kernel_stats.csv" > "$dest/summary_$(basename "$d").txt"
done
ls "$dest" | wc -l
