#!/bin/bash
# round 4: stride-2 split-f16 wgrad -- training gradient tests, wgrad_tr phase stamps, same-box
# training A/B (exact fp32-MFMA W0 wgrad vs wgrad_tr_kernel<XS_S2>)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/g_train.log 2>&1 || { tail -30 gpurun_out/g_train.log; exit 1; }
tail -2 gpurun_out/g_train.log
CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so timeout -k 10 200 python -u scripts/wgrad_stamps.py 8 > gpurun_out/wst.log 2>&1 || { tail -20 gpurun_out/wst.log; exit 1; }
cat gpurun_out/wst.log
for pass in 1 2; do
  for n in nos2 s2; do
    CISTA_HIP_LIB=v2e2v_amd/variants/$n.so timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abt_$n.json')); print(d['value'], d['ms_per_step'])")"
  done
done
