#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for a in none cpu_read sleep; do
  for i in 1 2; do run diag_${a}_$i 120 env PYTHONPATH=. python scripts/diag_replica_graph.py $a graph; done
done
run diag_cpu_read_eager 120 env PYTHONPATH=. python scripts/diag_replica_graph.py cpu_read eager
