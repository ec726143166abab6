#!/bin/bash
# Round-4 box (1/2): GPU tests + smoke + bench of the in-tree build; parity subset of every
# variant under v2e2v_amd/variants/ (vtests); same-box inference A/B over the variants.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests smoke bench vtests || exit $?
timeout -k 10 900 bash scripts/ab_bench.sh > gpurun_out/ab_bench.log 2>&1; rc=$?; cat gpurun_out/ab_bench.log; [ $rc -eq 0 ] || exit $rc
echo "r04b done"
