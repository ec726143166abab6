#!/bin/bash
# A/B of the tiled final-conv dgrad (CISTA_DFINAL_UNTILED=1: the round-4 kernel), training tests.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in tiled untiled; do
    if [ $v = untiled ]; then export CISTA_DFINAL_UNTILED=1; else unset CISTA_DFINAL_UNTILED; fi
    timeout -k 10 600 python bench.py --mode train --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/tb_$v.json 2> gpurun_out/tb_$v.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/tb_$v.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
unset CISTA_DFINAL_UNTILED
bash scripts/gpu_check.sh ttests tprof || exit $?
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/proft/run_kernel_stats.csv')))
for r in rows:
    if 'dgrad_final' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, 'us')
PY
