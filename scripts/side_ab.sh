set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ddp.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/side_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/side_tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do for side in 0 1; do
  CISTA_BWD_SIDE=$side timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/side_$side.json 2> gpurun_out/side_$side.err || exit $?
  echo "pass$pass side$side $(python -c "import json; d = json.load(open('gpurun_out/side_$side.json')); print(d['value'], d['ms_per_step'])")"
done; done
