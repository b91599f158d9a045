#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2; do
  run diag_before_$i 120 env PYTHONPATH=. MXDDP_REPLICA_SYNC=before python scripts/diag_replica_graph.py none graph
  run diag_after_$i 120 env PYTHONPATH=. MXDDP_REPLICA_SYNC=after python scripts/diag_replica_graph.py none graph
done
run diag_plain 120 env PYTHONPATH=. python scripts/diag_replica_graph.py none graph
