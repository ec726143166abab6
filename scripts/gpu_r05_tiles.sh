#!/bin/bash
# A/B of the dgrad tile ranking (CISTA_ZP2_HALO_W: 0 = pixel efficiency first, as round 4):
# training benches interleaved on one box, then the training tests on the default.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 0 0.25 0.5; do
    CISTA_ZP2_HALO_W=$w timeout -k 10 600 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline \
        > gpurun_out/tb_w$w.json 2> gpurun_out/tb_w$w.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/tb_w$w.json'));print('w=$w', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ddp.py -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/ttests.log 2>&1; rc=$?; echo "ttests rc=$rc"; tail -2 gpurun_out/ttests.log
