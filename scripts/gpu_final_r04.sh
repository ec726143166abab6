#!/bin/bash
# Round-4 validation on one GPU box, part 1 (every GPU step under its own time limit; a crash or
# timeout stops the script): GPU tests + smoke; the batch-bits diagnostic at B=48; PMC passes of
# the inference layers at the bench batch (FETCH_SIZE / WRITE_SIZE -> r04_pmc_traffic.json, SQ
# counters -> r04_pmc_counters.json), of the training step's dominant launch
# (-> r04_train_pmc_traffic.json) and of the layers at config c5's 720 x 1280
# (-> r04_v2e2v_pmc_traffic.json), copied under profiles/ so that the bench lines of part 2 quote
# this build's traffic.
set -o pipefail
bash scripts/gpu_check.sh tests smoke || exit $?
timeout -k 10 120 python scripts/diag_batch_bits.py 48 > gpurun_out/diag_bits_48.log 2>&1 || exit $?
echo "diag bits ok"; head -8 gpurun_out/diag_bits_48.log
bash scripts/pmc_layers.sh ${PMC_B:-256} || exit $?
python scripts/pmc_traffic.py 'gpurun_out/pmcl_*/run_counter_collection.csv' gpurun_out/r04_pmc_traffic.json > /dev/null || exit $?
python scripts/pmc_summary.py 'gpurun_out/pmcl_*/run_counter_collection.csv' > gpurun_out/r04_pmc_counters.json || exit $?
bash scripts/pmc_train_wgrad.sh || exit $?
python scripts/pmc_train_wgrad.py gpurun_out/r04_train_pmc_traffic.json > /dev/null || exit $?
bash scripts/pmc_v2e2v.sh 04 || exit $?
echo "final part 1 done"
