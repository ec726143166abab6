# HBM traffic of the CISTA layers at config c5's reconstruction size (720 x 1280, B = 1: the
# bench's --mode v2e2v line): FETCH_SIZE and WRITE_SIZE passes over scripts/layer_bench.py, one
# counter per pass, summarised into gpurun_out/rNN_v2e2v_pmc_traffic.json (usage: pmc_v2e2v.sh NN)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -f csv -d gpurun_out/pmcv2_$ctr -o run -- python3 scripts/layer_bench.py 1 720 1280 > gpurun_out/pmcv2_$ctr.out 2> gpurun_out/pmcv2_$ctr.err || exit $?
done
python scripts/pmc_traffic.py 'gpurun_out/pmcv2_*/run_counter_collection.csv' gpurun_out/r${1:-04}_v2e2v_pmc_traffic.json > /dev/null || exit $?
echo "pmc v2e2v ok"
