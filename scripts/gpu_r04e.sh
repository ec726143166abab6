#!/bin/bash
# Calibration of the overlap model: per-layer times at B=256 of the in-tree build vs one
# workgroup per CU (LDS-limited; no overlap between workgroups), two interleaved passes; and the
# phase timeline (CISTA_STAMPS=1 build) of the ISTA and gate convs at B=256.
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for f in v2e2v_amd/variants/base.so v2e2v_amd/exp/onewg.so; do
    CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py 256 >> gpurun_out/layerse.jsonl 2>> gpurun_out/layerse.err || exit $?
    echo "pass$pass $(basename $f) ok"
  done
done
CISTA_HIP_LIB=v2e2v_amd/exp/stamps.so timeout -k 10 300 python scripts/stamps.py 256 ista_D ista_P gates > gpurun_out/stamps256.jsonl 2> gpurun_out/stamps256.err || exit $?
cat gpurun_out/stamps256.jsonl
# training step A/B: in-tree vs two-tile-deep wgrad_tr staging (CISTA_WT_DEPTH=2), interleaved
for pass in 1 2; do
  for f in v2e2v_amd/variants/base.so v2e2v_amd/exp2/wtd2.so; do
    n=$(basename $f .so)
    CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abte_$n.json 2> gpurun_out/abte_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abte_$n.json')); print(d['value'], d['ms_per_step'])")"
  done
done
