#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r3*.sh one-offs):
#
#   scripts/gpu_run.sh <step> [<step> ...]
#
# Each step runs under its own timeout, logs to gpurun_out/<step>.log and appends to
# gpurun_out/steps.log; the run stops at the first crash / timeout (gpu_check.sh).  Kernel-trace
# summaries land in gpurun_out/summary_<step>.txt, counter passes in gpurun_out/pmc_<step>.txt.
# Steps:
#   suite        full GPU test suite (-x)      suite_all    the same, every failure reported
#   smoke        __graft_entry__.smoke()
#   t_<name>     one test file, tests/test_gpu_<name>.py      tsel   the pytest selection in $TSEL
#   driver       bench at the driver's length  long         2,000-step bench
#   prof_mnist   rocprofv3 kernel trace of the MNIST step
#   pmc_mnist    counter passes of the MNIST step (eager launches, one pass per run)
#   phase_mnist  in-kernel phase timings of the MNIST step
#   keras / keras_rep / keras_ws2 / prof_keras / pmc_keras   Keras CNN fused engine
#   mlp / mlp_rep / prof_mlp / pmc_mlp                       Chainer MLP
#   rn32 / rn256 / prof_rn / pmc_rn / rn_stock / rn_layers    ResNet-50 bf16 (rn_layers: per conv shape)
#   pyr / prof_pyr / pyr_stock                               PyramidNet-110
#   ws2 / ws4 / ws8 (MNIST), keras_ws8, pyr_ws8, rn_ws8      shared-GPU DDP rehearsals
#   coll         MNIST with RCCL collectives forced at one rank
#   cpu          BASELINE config 1
#   copies_pyr / copies_rn   torch.profiler census of the device copies in a layer-path step
#   trace_pyr    kernel + HIP API trace of the graphed PyramidNet step (where its copies come from)
#   diag_bnstats backward BN statistics of the data-gradient epilogues vs torch
#   bench_bn     effective bandwidth of the NHWC BN kernel variants vs a copy

source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log

SQ_A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ_B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"

prof() {  # prof <name> <steps-for-per-step-numbers> <bench args...>
  local name=$1 n=$2; shift 2
  run "$name" 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o run --output-format csv -- python bench.py "$@"
  python scripts/kstats.py "$(find "gpurun_out/$name" -name '*kernel_stats.csv' | head -1)" "$n" > "gpurun_out/summary_$name.txt" || true
}
pmc() {  # pmc <name> <bench args...>: 4 counter passes (SQ A, SQ B, FETCH_SIZE, WRITE_SIZE)
  local name=$1; shift
  local i=0
  for set in "$SQ_A" "$SQ_B" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    run "${name}_$i" 90 timeout -s KILL 80 rocprofv3 --pmc $set --kernel-trace --output-format csv \
      -d "gpurun_out/${name}_$i" -o run -- python bench.py "$@"
  done
  python scripts/pmc_summary.py $(find gpurun_out/${name}_[1-4] -name '*counter_collection.csv') > "gpurun_out/$name.txt" || true
}
ws() {  # ws <name> <ranks> <bench args...>: ranks share the one GPU (functional rehearsal)
  local name=$1 n=$2; shift 2
  run "$name" 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 400)) bench.py --gpus "$n" "$@"
}

for step in "$@"; do
  case "$step" in
    suite) run suite 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    suite_all) run suite_all 1500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    tsel) run tsel 900 python -u -m pytest ${TSEL:?set TSEL to the pytest selection} -m gpu -v --timeout 120 --timeout-method thread ;;
    t_*) run "$step" 900 python -u -m pytest "tests/test_gpu_${step#t_}.py" -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) run driver 300 python bench.py --steps 20 --warmup 5 ;;
    driver_all)  # every fused model at the driver's length, and the 2-rank rehearsal
      run driver_mnist 300 python bench.py --steps 20 --warmup 5 &&
      run driver_keras 300 python bench.py --model keras_cnn --steps 20 --warmup 5 &&
      run driver_mlp 300 python bench.py --model mlp --steps 20 --warmup 5 || exit 1
      ws driver_ws2 2 --steps 20 --warmup 5 ;;
    long) run long 300 python bench.py --steps 2000 --warmup 100 ;;
    default) run default 300 python bench.py ;;
    prof_mnist) prof prof_mnist 200 --steps 200 --warmup 20 --min-warmup-ms 0 ;;
    pmc_mnist) pmc pmc_mnist --steps 20 --warmup 2 --no-graph --min-warmup-ms 0 ;;
    phase_mnist) run phase_mnist 300 python bench.py --phase-profile 30 ;;
    bench_bn) run bench_bn 300 python scripts/bench_bn.py ;;
    coll) run coll 300 python bench.py --steps 2000 --warmup 100 --force-collectives ;;
    replica) run replica 300 python bench.py --impl replica --steps 1000 --warmup 50 ;;
    layers) run layers 300 python bench.py --impl layers --steps 300 --warmup 30 ;;
    cpu) run cpu 300 python bench.py --cpu --steps 30 --warmup 3 ;;
    keras) run keras 300 python bench.py --model keras_cnn --steps 2000 --warmup 100 ;;
    keras_rep) run keras_rep 300 python bench.py --model keras_cnn --impl replica --steps 1000 --warmup 50 ;;
    prof_keras) prof prof_keras 200 --model keras_cnn --steps 200 --warmup 20 --min-warmup-ms 0 ;;
    pmc_keras) pmc pmc_keras --model keras_cnn --steps 20 --warmup 2 --no-graph --min-warmup-ms 0 ;;
    mlp) run mlp 300 python bench.py --model mlp --steps 2000 --warmup 100 ;;
    mlp_layers) run mlp_layers 300 python bench.py --model mlp --impl layers --steps 300 --warmup 30 ;;
    mlp_rep) run mlp_rep 300 python bench.py --model mlp --impl replica --steps 1000 --warmup 50 ;;
    prof_mlp) prof prof_mlp 200 --model mlp --steps 200 --warmup 20 --min-warmup-ms 0 ;;
    pmc_mlp) pmc pmc_mlp --model mlp --steps 20 --warmup 2 --no-graph --min-warmup-ms 0 ;;
    rn32) run rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 ;;
    rn256) run rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3 ;;
    rn_layers) run rn_layers 300 python scripts/bench_nhwc_layers.py 256 5 ;;
    rn_stock) run rn_stock 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3 --impl torch --channels-last ;;
    prof_rn32) prof prof_rn32 10 --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 2 --min-warmup-ms 0 ;;
    prof_rn) prof prof_rn 3 --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2 --min-warmup-ms 0 ;;
    prof_rn_stock) prof prof_rn_stock 3 --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2 --min-warmup-ms 0 --impl torch --channels-last ;;
    pmc_rn) pmc pmc_rn --model resnet50 --dtype bf16 --batch 256 --steps 1 --warmup 1 --no-graph --min-warmup-ms 0 ;;
    pyr) run pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3 ;;
    pyr_stock) run pyr_stock 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3 --impl torch ;;
    pmc_pyr) pmc pmc_pyr --model pyramidnet110 --steps 1 --warmup 1 --no-graph --min-warmup-ms 0 ;;
    prof_pyr) prof prof_pyr 5 --model pyramidnet110 --steps 5 --warmup 2 --min-warmup-ms 0 ;;
    prof_pyr_stock) prof prof_pyr_stock 5 --model pyramidnet110 --steps 5 --warmup 2 --min-warmup-ms 0 --impl torch ;;
    ws2) ws ws2 2 --steps 1000 --warmup 50 ;;
    ws4) ws ws4 4 --steps 500 --warmup 20 ;;
    ws8) ws ws8 8 --steps 200 --warmup 20 ;;
    ws8_driver) ws ws8_driver 8 --steps 20 --warmup 5 ;;   # the driver's exact 8-rank command
    ab)  # one A/B pass: AB="bench args" (e.g. AB="--model resnet50 --dtype bf16 --batch 32 --ab wgrad_target=256")
      run ab 300 python bench.py ${AB:?set AB to the bench arguments} ;;
    keras_ws2) ws keras_ws2 2 --model keras_cnn --steps 300 --warmup 30 ;;
    keras_ws8) ws keras_ws8 8 --model keras_cnn --steps 100 --warmup 10 ;;
    pyr_ws8) ws pyr_ws8 8 --model pyramidnet110 --batch 8 --steps 5 --warmup 2 ;;
    rn_ws8) ws rn_ws8 8 --model resnet50 --dtype bf16 --batch 8 --steps 5 --warmup 2 ;;
    trace_pyr) run trace_pyr 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/trace_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --steps 3 --warmup 2 --min-warmup-ms 0 ;;
    diag_bnstats) run diag_bnstats 300 python scripts/diag_bn_dgrad_stats.py ;;
    copies_pyr) run copies_pyr 300 python scripts/diag_copies.py pyramidnet110 fp32 64 ;;
    copies_rn) run copies_rn 300 python scripts/diag_copies.py resnet50 bf16 32 ;;
    *) echo "gpu_run.sh: unknown step $step"; exit 2 ;;
  esac
done
