# One training step: the LDS counters of the split-f16 wgrad (and every other kernel) in one pass
set -o pipefail
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -f csv -d gpurun_out/pmcw -o run -- python3 bench.py --mode train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcw.out 2> gpurun_out/pmcw.err
