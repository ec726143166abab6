cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/vprof -o run -- python3 scripts/vox_prof.py 960 5 > gpurun_out/vprof.json 2> gpurun_out/vprof.err || exit $?
bash scripts/pmc_layers.sh 64 || exit $?
echo done
