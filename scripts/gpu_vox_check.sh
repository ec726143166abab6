# voxelizer: GPU parity tests, the 960-window call timed (HIP events), rocprof kernel statistics
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py tests/test_gpu_v2e.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vox_tests.log 2>&1; rc=$?; tail -3 gpurun_out/vox_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/vox_prof.py 960 10 > gpurun_out/vox_new.json && cat gpurun_out/vox_new.json || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/vprof2 -o run -- python3 scripts/vox_prof.py 960 5 > /dev/null 2>&1 || exit $?
echo done
