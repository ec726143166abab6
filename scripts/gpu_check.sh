#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench (-> optional rocprof).  Every GPU step has
# its own time limit; after a crash / fault / timeout nothing else touches the GPU.
# usage: bash scripts/gpu_check.sh [tests] [smoke] [bench] [prof] [ttests] [tbench] [tprof] [vbench] [vprof] [pmc] ...
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures, not a crash
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sweep "" > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.err; [ $rc -eq 0 ] || exit $rc ;;
    ttests)
      timeout -k 10 600 python -m pytest tests/test_gpu_train.py -m gpu -q -p no:cacheprovider > gpurun_out/gpu_ttests.log 2>&1
      rc=$?; echo "ttests rc=$rc"; tail -12 gpurun_out/gpu_ttests.log; ok $rc || exit $rc ;;
    tbench)
      timeout -k 10 600 python bench.py --mode train ${TBENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/tbench.json 2> gpurun_out/tbench.err
      rc=$?; echo "tbench rc=$rc"; cat gpurun_out/tbench.json; tail -3 gpurun_out/tbench.err; [ $rc -eq 0 ] || exit $rc ;;
    vbench)
      timeout -k 10 600 python bench.py --mode v2e2v ${VBENCH_ARGS:---steps 2 --warmup 1} > gpurun_out/vbench.json 2> gpurun_out/vbench.err
      rc=$?; echo "vbench rc=$rc"; cat gpurun_out/vbench.json; tail -3 gpurun_out/vbench.err; [ $rc -eq 0 ] || exit $rc ;;
    tprof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/proft -o run -- python3 bench.py --mode train --steps 1 --warmup 1 > gpurun_out/proft_bench.json 2> gpurun_out/proft.err
      rc=$?; echo "tprof rc=$rc"; tail -3 gpurun_out/proft.err; [ $rc -eq 0 ] || exit $rc ;;
    vprof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/profv -o run -- python3 bench.py --mode v2e2v --steps 1 --warmup 1 > gpurun_out/profv_bench.json 2> gpurun_out/profv.err
      rc=$?; echo "vprof rc=$rc"; tail -3 gpurun_out/profv.err; [ $rc -eq 0 ] || exit $rc ;;
    ab)
      timeout -k 10 900 bash scripts/ab_layers.sh ${AB_B:-64}
      rc=$?; echo "ab rc=$rc"; cat gpurun_out/layers.jsonl; [ $rc -eq 0 ] || exit $rc ;;
    list)
      timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?" ;;
    sq)
      timeout -k 10 600 rocprofv3 --pmc ${SQ_CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT} --kernel-trace -f csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --layer-reps 3 > /dev/null 2> gpurun_out/pmc_sq.err
      rc=$?; echo "sq rc=$rc"; tail -2 gpurun_out/pmc_sq.err; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -f csv -d gpurun_out/pmc_$ctr -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --layer-reps 3 > /dev/null 2> gpurun_out/pmc_$ctr.err
        rc=$?; echo "pmc $ctr rc=$rc"; tail -2 gpurun_out/pmc_$ctr.err; [ $rc -eq 0 ] || exit $rc
      done ;;
  esac
done
