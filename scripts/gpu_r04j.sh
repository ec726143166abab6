#!/bin/bash
# round 4: register-weight final-conv dgrad (dgrad_final_rows_kernel) -- training tests, per-kernel
# times and a same-box training A/B; wgrad_tr with idle staging waves (timing experiment)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/j_train.log 2>&1 || { tail -40 gpurun_out/j_train.log; exit 1; }
tail -1 gpurun_out/j_train.log
CISTA_HIP_LIB=v2e2v_amd/variants/stidle.so timeout -k 10 200 python -u scripts/wgrad_stamps.py 8 > gpurun_out/wst_stidle.log 2>&1 || exit 1
echo stidle; tail -1 gpurun_out/wst_stidle.log
for n in dfold dfrows; do
  CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abj_$n -o run -- python3 bench.py --mode train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abj_$n.out 2>&1 || exit $?
  echo "$n $(grep -E 'dgrad_final|wgrad_tr' gpurun_out/abj_$n/run_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
for pass in 1 2; do
  for n in dfold dfrows; do
    CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abt_$n.json')); print(d['value'], d['ms_per_step'])")"
  done
done
