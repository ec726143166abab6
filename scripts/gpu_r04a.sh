#!/bin/bash
# Round-4 box: GPU tests, smoke, bench; the DVFS probe (He-init vs zero weights per layer); a
# same-box A/B of the training step over v2e2v_amd/variants/*.so; a per-launch kernel trace of
# one training step.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests smoke bench || exit $?
timeout -k 10 300 python scripts/power_probe.py 256 gpurun_out/power_probe.json > gpurun_out/power_probe.log 2>&1 || exit $?
echo "power probe ok"
bash scripts/ab_train.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace_train -o run -- python3 bench.py --mode train --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/trace_train.json 2> gpurun_out/trace_train.err || exit $?
echo "train trace ok"
