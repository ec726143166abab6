# Round-end validation on one GPU box: GPU tests, smoke, the default bench line, rocprof kernel
# statistics of the bench, the training bench and the V2E2V bench, PMC passes at the bench batch,
# and the bench under torchrun (N=1: the rendezvous / barrier / max-over-ranks path the driver's
# multi-GPU runs take).  Each GPU step has its own time limit; a crash or timeout stops the script.
set -o pipefail
bash scripts/gpu_check.sh tests smoke bench prof tbench tprof vbench vprof || exit $?
bash scripts/pmc_layers.sh ${PMC_B:-256} || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --sweep= \
    > gpurun_out/torchrun.json 2> gpurun_out/torchrun.err || exit $?
echo "torchrun ok"; cut -c1-200 gpurun_out/torchrun.json
echo final done
