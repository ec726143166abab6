#!/bin/bash
# Round-6 validation on one GPU box, part 1 (every GPU step under its own time limit; a crash or
# timeout stops the script): GPU tests + smoke; PMC passes of the inference layers at the bench
# batch (FETCH_SIZE / WRITE_SIZE -> r06_pmc_traffic.json, SQ counters -> r06_pmc_counters.json),
# of the training step's dominant launch (-> r06_train_pmc_traffic.json) and of the layers at
# config c5's 720 x 1280 (-> r06_v2e2v_pmc_traffic.json), copied under profiles/ so that the bench
# lines of part 2 quote this build's traffic.
set -o pipefail
bash scripts/gpu_check.sh tests smoke || exit $?
rm -rf gpurun_out/pmcl_* gpurun_out/pmctw_* gpurun_out/pmcv2_*
bash scripts/pmc_layers.sh ${PMC_B:-256} || exit $?
python scripts/pmc_traffic.py 'gpurun_out/pmcl_*/run_counter_collection.csv' gpurun_out/r06_pmc_traffic.json > /dev/null || exit $?
python scripts/pmc_summary.py 'gpurun_out/pmcl_*/run_counter_collection.csv' > gpurun_out/r06_pmc_counters.json || exit $?
bash scripts/pmc_train_wgrad.sh || exit $?
python scripts/pmc_train_wgrad.py gpurun_out/r06_train_pmc_traffic.json > /dev/null || exit $?
bash scripts/pmc_v2e2v.sh 06 || exit $?
echo "final part 1 done"
