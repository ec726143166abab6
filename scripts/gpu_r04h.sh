#!/bin/bash
# round 4: W0 stride-2 wgrad test hook + split counts of the small VALU wgrads (per-kernel times
# from rocprofv3 kernel-trace stats of a 2-step training bench per variant)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 200 --timeout-method thread -m gpu -k "wgrad" > gpurun_out/h_train.log 2>&1 || { tail -30 gpurun_out/h_train.log; exit 1; }
tail -2 gpurun_out/h_train.log
for n in ns512 ns1k ns2k; do
  CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abk_$n -o run -- python3 bench.py --mode train --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abk_$n.out 2>&1 || exit $?
  f=$(find gpurun_out/abk_$n -name "run_kernel_stats.csv" | head -1)
  echo "$n $(grep -E 'wgrad_small|wgrad_c1' $f | cut -d, -f1-4 | tr '\n' ' ')"
done
