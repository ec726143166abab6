# end-to-end inference A/B of every build under v2e2v_amd/variants/ (one process per build,
# the list run twice in alternating order to expose box drift)
for pass in 1 2; do
  for f in v2e2v_amd/variants/*.so; do
    n=$(basename $f .so)
    CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/ab_$n.json')); print(d['value'], d['layers_ms'].get('input', d['layers_ms'].get('input+W0')), d['layers_ms'].get('W0'))")"
  done
done
