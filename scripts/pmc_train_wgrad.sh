# PMC passes over the training step's dominant launch alone (scripts/train_wgrad_bench.py):
# FETCH_SIZE and WRITE_SIZE in passes of their own, then the SQ / GRBM counters; summarised by
# scripts/pmc_train_wgrad.py into profiles/rNN_train_pmc_traffic.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d gpurun_out/pmctw_$i -o run -- python3 scripts/train_wgrad_bench.py 6 > gpurun_out/pmctw_$i.out 2> gpurun_out/pmctw_$i.err || exit $?
done
