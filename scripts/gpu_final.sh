# Round-end validation on one GPU box: GPU tests, smoke, the default bench line, rocprof kernel
# statistics of the bench and the training bench, PMC passes at the bench batch.  Each GPU step
# has its own time limit; a crash or timeout stops the script.
set -o pipefail
bash scripts/gpu_check.sh tests smoke bench prof tbench tprof || exit $?
bash scripts/pmc_layers.sh ${PMC_B:-256} || exit $?
echo final done
