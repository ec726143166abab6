#!/bin/bash
# round 4: fused We / Wi wgrad (wgrad_in_kernel) -- training gradient tests, per-kernel times
# (rocprofv3 kernel-trace stats) and a same-box training A/B against the two wgrad_small launches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/i_train.log 2>&1 || { tail -40 gpurun_out/i_train.log; exit 1; }
tail -2 gpurun_out/i_train.log
for n in win0 win1; do
  CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abi_$n -o run -- python3 bench.py --mode train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abi_$n.out 2>&1 || exit $?
  f=$(find gpurun_out/abi_$n -name "run_kernel_stats.csv" | head -1)
  echo "$n $(grep -E 'wgrad_small|wgrad_in|dgrad_c1' $f | cut -d, -f1-4 | tr '\n' ' ')"
done
for pass in 1 2; do
  for n in win0 win1; do
    CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abt_$n.json')); print(d['value'], d['ms_per_step'])")"
  done
done
