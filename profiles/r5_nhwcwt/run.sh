set -e
O=gpurun_out/wt2
mkdir -p $O
for r in 1 2 3; do
  for v in base both; do
    args=""; [ $v = both ] && args="--ab bn_wt=1 --ab conv_wt=1"
    timeout -k 10 200 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 20 --warmup 3 $args > $O/rn256_${v}_$r.log 2>&1
    timeout -k 10 200 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 30 --warmup 5 $args > $O/rn32_${v}_$r.log 2>&1
    timeout -k 10 200 python bench.py --model pyramidnet110 --dtype bf16 --batch 128 --steps 20 --warmup 3 $args > $O/pyr_${v}_$r.log 2>&1
  done
done
