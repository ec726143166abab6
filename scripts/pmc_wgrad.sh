# One training step: MFMA-busy, LDS and wait counters of every kernel (the split-f16 wgrad first
# of all) in one rocprofv3 pass (8 SQ + 1 GRBM counters)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d gpurun_out/pmcw -o run -- python3 bench.py --mode train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcw.out 2> gpurun_out/pmcw.err
