# PMC passes over one training step (bench.py --mode train), one counter group per pass, kernel
# trace only; summarise with: python scripts/pmc_summary.py 'gpurun_out/pmct_*/run_counter_collection.csv'
set -o pipefail
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d gpurun_out/pmct_$i -o run -- python3 bench.py --mode train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmct_$i.out 2> gpurun_out/pmct_$i.err || exit $?
done
echo pmc train done
