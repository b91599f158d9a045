#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2 3; do
  run diag_noalloc_$i 120 env PYTHONPATH=. python scripts/diag_replica_graph.py noalloc graph
done
run diag_none 120 env PYTHONPATH=. python scripts/diag_replica_graph.py none graph
