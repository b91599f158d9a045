#!/bin/bash
# Round-end evidence on one MI355X: the full GPU suite, smoke, the driver's bench and a long run,
# kernel traces of the MNIST / Keras / MLP / ResNet-50 / PyramidNet steps, the secondary benches
# and the shared-GPU DDP rehearsals.  Logs under gpurun_out/ (copy to profiles/<round>_final/).
"$(dirname "$0")/gpu_run.sh" suite smoke driver long default prof_mnist keras keras_rep prof_keras \
  mlp mlp_rep prof_mlp rn32 rn256 prof_rn pyr prof_pyr cpu replica coll ws2 keras_ws2
