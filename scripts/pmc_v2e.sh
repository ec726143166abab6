# Emulator at config c5's size (scripts/v2e_prof.py): kernel trace, then PMC passes, one counter
# group per pass; summarise with: python scripts/pmc_summary.py 'gpurun_out/pmcv_*/run_counter_collection.csv'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/v2etr -o run -- python3 scripts/v2e_prof.py 4 > gpurun_out/v2etr.out 2>&1 || exit $?
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d gpurun_out/pmcv_$i -o run -- python3 scripts/v2e_prof.py 2 > gpurun_out/pmcv_$i.out 2>&1 || exit $?
done
echo pmc v2e done
