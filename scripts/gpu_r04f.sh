#!/bin/bash
# A/B: in-tree vs chunk-1 halo + chunk-0 B taps issued in the prologue (CISTA_HOIST1=1): per-layer
# times at B=256 and the end-to-end bench, interleaved over two passes; parity subset of the variant
set -o pipefail
mkdir -p gpurun_out
CISTA_HIP_LIB=v2e2v_amd/exp2/hoist.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider -k "stage or f3 or oracle_random or f1_sequence or batch" > gpurun_out/vtests_hoist.log 2>&1; rc=$?; tail -1 gpurun_out/vtests_hoist.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for f in v2e2v_amd/variants/base.so v2e2v_amd/exp2/hoist.so; do
    n=$(basename $f .so)
    CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py 256 >> gpurun_out/layersf.jsonl 2>> gpurun_out/layersf.err || exit $?
    CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sweep= > gpurun_out/abf_$n.json 2> gpurun_out/abf_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abf_$n.json')); print(d['value'])")"
  done
done
# timing-only: ISTA P writing z out of place (results wrong by design)
for pass in 1 2; do
  for f in v2e2v_amd/variants/base.so v2e2v_amd/exp3/zout.so; do
    CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py 256 >> gpurun_out/layersz.jsonl 2>> gpurun_out/layersz.err || exit $?
  done
done
echo "zout done"
