#!/bin/bash
# Round-6 validation, part 2 (profiles/r06_*_pmc_traffic.json of this build committed first): the
# bench lines with their rocprofv3 kernel statistics, and the benches under torchrun at N=1 (the
# driver's multi-GPU path: one RCCL rank; training wraps the model in DDP), then the conv phase
# timeline of a CISTA_STAMPS=1 build of the same sources.
set -o pipefail
bash scripts/gpu_check.sh bench prof tbench tprof vbench vprof || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --sweep= \
    > gpurun_out/torchrun.json 2> gpurun_out/torchrun.err || exit $?
echo "torchrun ok"; cut -c1-200 gpurun_out/torchrun.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --mode train --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/torchrun_train.json 2> gpurun_out/torchrun_train.err || exit $?
echo "torchrun train ok"; cut -c1-200 gpurun_out/torchrun_train.json
CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so timeout -k 10 300 python scripts/stamps.py 256 ista_D ista_P gates lstm out_gates \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err || exit $?
echo "stamps ok"
echo final done
