#!/bin/bash
# Round-5 iteration box: GPU tests + smoke + bench of the in-tree build; the ISTA P L2-window
# probe (timing, then its held clock under a GRBM_GUI_ACTIVE pass); SQ instruction counters of the
# layers at the bench batch.  Every GPU step under its own time limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh ${CHECK_STEPS:-tests smoke bench} || exit $?
export TMPDIR=/tmp
CISTA_HIP_LIB=v2e2v_amd/variants/probe.so timeout -k 10 300 python scripts/l2_probe.py 256 100 gpurun_out/l2_probe.json \
    > gpurun_out/l2_probe.log 2>&1 || exit $?
echo "l2 probe ok"; cat gpurun_out/l2_probe.json
CISTA_HIP_LIB=v2e2v_amd/variants/probe.so timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
    --kernel-trace -f csv -d gpurun_out/pmc_probe -o run -- python3 scripts/l2_probe.py 256 20 gpurun_out/l2_probe_pmc.json \
    > gpurun_out/pmc_probe.log 2>&1 || exit $?
echo "l2 probe pmc ok"
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d gpurun_out/pmcl_$i -o run -- python3 scripts/layer_bench.py 256 \
      > gpurun_out/pmcl_$i.out 2> gpurun_out/pmcl_$i.err || exit $?
  echo "pmc pass $i ok"
done
python scripts/pmc_summary.py 'gpurun_out/pmcl_*/run_counter_collection.csv' > gpurun_out/r05_pmc_counters.json || exit $?
echo iter done
