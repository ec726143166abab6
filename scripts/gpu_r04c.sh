#!/bin/bash
# Round-4 box (2/2): per-layer HIP-event times at B=256 of the in-tree build, the persistent
# variant and three timing-only experiment builds (wrong results by design: stores wrapped into a
# 16 KB window / epilogue stores skipped / halo staged only for the first K-chunk); the DVFS probe;
# the training A/B over v2e2v_amd/variants/ and a per-launch kernel trace of one training step.
set -o pipefail
mkdir -p gpurun_out
for bb in 48 32; do
  timeout -k 10 120 python scripts/diag_batch_bits.py $bb > gpurun_out/diag_bits_$bb.log 2>&1 || exit $?
done
echo "diag bits ok"; cat gpurun_out/diag_bits_48.log
for f in v2e2v_amd/variants/base.so v2e2v_amd/variants/pers.so v2e2v_amd/exp/smallst.so v2e2v_amd/exp/noepi.so v2e2v_amd/exp/nostage.so; do
  CISTA_HIP_LIB=$f timeout -k 10 300 python scripts/layer_bench.py 256 >> gpurun_out/layers256.jsonl 2>> gpurun_out/layers256.err || exit $?
  echo "layers $(basename $f) ok"
done
timeout -k 10 300 python scripts/power_probe.py 256 gpurun_out/power_probe.json > gpurun_out/power_probe.log 2>&1 || exit $?
echo "power probe ok"
bash scripts/ab_train.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace_train -o run -- python3 bench.py --mode train --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/trace_train.json 2> gpurun_out/trace_train.err || exit $?
echo "r04c done"
