for pass in 1 2; do
  for f in v2e2v_amd/variants/*.so; do
    n=$(basename $f .so)
    CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --sweep= > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/ab_$n.json')); print(d['value'], d['sum_of_kernels_ms_per_frame_batch'], d['layers_ms'])")"
  done
done
