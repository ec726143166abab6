#!/bin/bash
# A/B of per-layer HIP-event times at B=256, interleaved over two passes: the in-tree build vs
# the MFMA issue-order variant (and any other build under v2e2v_amd/exp/)
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for f in v2e2v_amd/variants/base.so v2e2v_amd/exp/*.so; do
    CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py 256 >> gpurun_out/layersd.jsonl 2>> gpurun_out/layersd.err || exit $?
    echo "pass$pass $(basename $f) ok"
  done
done
