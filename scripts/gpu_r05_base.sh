#!/bin/bash
# Round-5 first box: GPU tests + smoke, the inference and training bench lines, and the
# training bench under torchrun at N=1 (one RCCL rank, DDP all-reduce: "parallelism": "ddp1").
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests smoke bench tbench || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --mode train --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/torchrun_train.json 2> gpurun_out/torchrun_train.err || exit $?
echo "torchrun train ok"; cut -c1-400 gpurun_out/torchrun_train.json
