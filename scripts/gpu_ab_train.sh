#!/bin/bash
# same-box A/B of the BPTT training bench over the named builds in v2e2v_amd/variants/ (interleaved passes)
# usage: bash scripts/gpu_ab_train.sh passes name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
np=$1; shift
for pass in $(seq 1 $np); do
  for n in "$@"; do
    CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abt_$n.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'])")"
  done
done
