#!/bin/bash
# A/B of this round's conv changes: parity + batch-invariance tests on the in-tree build and on
# the variants (no aux prefetch, library gate functions), inference and training benches of each,
# then the phase stamps.  Every GPU step under its own limit; the first crash ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/diag_batch_bits.py 48 > gpurun_out/diag_bits_48.log 2>&1 || exit $?
echo "diag bits ok"; head -12 gpurun_out/diag_bits_48.log
for lib in v2e2v_amd/libcista_hip.so v2e2v_amd/variants/nopref.so v2e2v_amd/variants/slowgates.so; do
  n=$(basename $lib .so)
  CISTA_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/bits_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc"; tail -2 gpurun_out/bits_$n.log; [ $rc -le 1 ] || exit $rc
done
for lib in v2e2v_amd/libcista_hip.so v2e2v_amd/variants/nopref.so v2e2v_amd/variants/slowgates.so; do
  n=$(basename $lib .so)
  CISTA_HIP_LIB=$lib timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --sweep= \
      > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_$n.json'));print('$n', d['value'], d['max_elementwise_rel_err_vs_ref'], d['layers_ms'])"
  CISTA_HIP_LIB=$lib timeout -k 10 600 python bench.py --mode train --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/tbench_$n.json 2> gpurun_out/tbench_$n.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/tbench_$n.json'));print('$n train', d['value'])"
done
CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so timeout -k 10 300 python scripts/stamps.py 256 ista_D ista_P gates lstm out_gates \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err || exit $?
echo stamps ok; cat gpurun_out/stamps.json
