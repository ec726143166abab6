#!/bin/bash
# Training A/B of the Adam implementation (fused vs foreach), interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for a in foreach fused; do
    timeout -k 10 600 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline --adam $a \
        > gpurun_out/adam_$a.json 2> gpurun_out/adam_$a.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/adam_$a.json'));print('$a', d['value'], d['ms_per_step'], d['loss'])"
  done
done
