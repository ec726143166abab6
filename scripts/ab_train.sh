# training-step A/B of every build under v2e2v_amd/variants/ (one process per build)
for f in v2e2v_amd/variants/*.so; do
  n=$(basename $f .so)
  CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --mode train --steps 3 --warmup 1 > gpurun_out/tb_$n.json 2> gpurun_out/tb_$n.err || exit $?
  echo "$n $(python -c "import json; d = json.load(open('gpurun_out/tb_$n.json')); print(d['value'], d['ms_per_step'])")"
done
