#!/bin/bash
# Same-box A/B of the stacked ISTA P wgrad launch (scripts/train_wgrad_bench.py) over the libraries
# in v2e2v_amd/variants/: HIP-event launch time (3 interleaved passes), then the HBM bytes of each
# arm (FETCH_SIZE / WRITE_SIZE passes of their own), then the training bench (scripts/ab_train.sh).
# Writes gpurun_out/wt_ab.txt and gpurun_out/wtpmc_<arm>_<counter>/.  The round-6 arms were built
# from commit 8ce774e (build_variants.sh wt_blk "-DCISTA_WT_XCD=0" wt_xcd "-DCISTA_WT_XCD=1"); the
# switch is gone since, so at later commits any two libraries can be compared this way.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pass in 1 2 3; do
  for f in v2e2v_amd/variants/*.so; do
    n=$(basename $f .so)
    r=$(CISTA_HIP_LIB=$f timeout -k 10 120 python scripts/train_wgrad_bench.py 20 2> gpurun_out/wt_$n.err) || exit $?
    echo "pass$pass $n $r" | tee -a gpurun_out/wt_ab.txt
  done
done
for f in v2e2v_amd/variants/*.so; do
  n=$(basename $f .so)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    CISTA_HIP_LIB=$f timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -f csv -d gpurun_out/wtpmc_${n}_$ctr -o run \
      -- python3 scripts/train_wgrad_bench.py 6 > /dev/null 2> gpurun_out/wtpmc_${n}_$ctr.err || exit $?
    echo "pmc $n $ctr done" | tee -a gpurun_out/wt_ab.txt
  done
done
[ -n "$WT_TRAIN" ] && { bash scripts/ab_train.sh | tee -a gpurun_out/wt_ab.txt || exit $?; }
exit 0
