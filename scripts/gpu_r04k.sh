#!/bin/bash
# round 4: validation of the wgrad_tr staging changes -- full GPU suite, training bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/k_tests.log 2>&1 || { tail -40 gpurun_out/k_tests.log; exit 1; }
tail -1 gpurun_out/k_tests.log
for pass in 1 2; do
  timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/k_train.json 2> gpurun_out/k_train.err || exit $?
  echo "pass$pass $(python -c "import json; d = json.load(open('gpurun_out/k_train.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])")"
done
