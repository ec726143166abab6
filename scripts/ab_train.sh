# Same-box A/B of the BPTT training bench over the libraries in v2e2v_amd/variants/ (two passes,
# interleaved, so box-to-box variance does not enter the comparison)
for pass in 1 2; do
  for f in v2e2v_amd/variants/*.so; do
    n=$(basename $f .so)
    CISTA_HIP_LIB=$f timeout -k 10 300 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || exit $?
    echo "pass$pass $n $(python -c "import json; d = json.load(open('gpurun_out/abt_$n.json')); print(d['value'], d['ms_per_step'])")"
  done
done
