#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2; do
  run diag_none_$i 120 env PYTHONPATH=. python scripts/diag_replica_graph.py none graph
  run diag_side_$i 120 env PYTHONPATH=. MXDDP_REPLICA_REPLAY_SIDE=1 python scripts/diag_replica_graph.py none graph
  run diag_blocking_$i 120 env PYTHONPATH=. AMD_SERIALIZE_KERNEL=3 python scripts/diag_replica_graph.py none graph
done
