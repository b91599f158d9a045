#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run diag_long 120 env PYTHONPATH=. python scripts/diag_replica_graph.py long graph
run diag_none 120 env PYTHONPATH=. python scripts/diag_replica_graph.py none graph
run diag_long_eager 120 env PYTHONPATH=. python scripts/diag_replica_graph.py long eager
