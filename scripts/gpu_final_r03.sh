# Round-3 validation on one GPU box (every GPU step under its own time limit; a crash or timeout
# stops the script): GPU tests + smoke; PMC passes of the inference layers at the bench batch
# (FETCH_SIZE / WRITE_SIZE -> r03_pmc_traffic.json, SQ counters -> r03_pmc_counters.json) and
# of the training step's dominant launch (-> r03_train_pmc_traffic.json), copied under profiles/
# so that the bench lines below quote this build's traffic; then the bench lines with their
# rocprofv3 kernel statistics, and the bench under torchrun (N=1: the driver's multi-GPU path).
set -o pipefail
bash scripts/gpu_check.sh tests smoke || exit $?
bash scripts/pmc_layers.sh ${PMC_B:-256} || exit $?
python scripts/pmc_traffic.py 'gpurun_out/pmcl_*/run_counter_collection.csv' gpurun_out/r03_pmc_traffic.json > /dev/null || exit $?
python scripts/pmc_summary.py 'gpurun_out/pmcl_*/run_counter_collection.csv' > gpurun_out/r03_pmc_counters.json || exit $?
bash scripts/pmc_train_wgrad.sh || exit $?
python scripts/pmc_train_wgrad.py gpurun_out/r03_train_pmc_traffic.json > /dev/null || exit $?
cp gpurun_out/r03_pmc_traffic.json gpurun_out/r03_train_pmc_traffic.json profiles/ || exit $?
echo "pmc ok"
bash scripts/gpu_check.sh bench prof tbench tprof vbench vprof || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --sweep= \
    > gpurun_out/torchrun.json 2> gpurun_out/torchrun.err || exit $?
echo "torchrun ok"; cut -c1-200 gpurun_out/torchrun.json
echo final done
